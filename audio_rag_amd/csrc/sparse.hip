// Sparse lexical-weight top-k over a device inverted index (gfx950).
//
// Restates Qdrant's sparse-vector search as called by QdrantRetriever.search
// (src/audio_rag/retrieval/qdrant.py:289-293 sparse prefetch of hybrid search, 299-312 sparse
// query) on the collection's "sparse" vector (SparseVectorParams without IDF modifier,
// qdrant.py:103-107), filled with BGE-M3 lexical weights (embeddings/bge.py:95-102, 122-128):
//   score(q, d) = sum over indices present in both, in ascending index order, of fl32(q_i * d_i)
//   accumulated in fp32 (multiply and add rounded separately; no FMA), only rows that share at
//   least one index are results, ranking (score desc, ordinal asc).
//
// Layout (built on the device at create time): postings per term, ascending row, each list
// closed by a sentinel row; rows cut into one contiguous range per CU.
//
// Search, one pass per 64 queries:
//   pass_terms: the 64 queries are dealt to 16 waves, 4 each (slot 4w + i), and every slot gets
//           the ascending list of its query's terms as (staging row offset, weight).
//   scan:   workgroup = one row range, wave = 4 queries, lane = four adjacent rows of a 256-row
//           tile. Each distinct term of the pass is staged once per tile: its holder wave loads
//           the next 128 postings (lane-reversed; more while the tile holds more), keeps the
//           prefix inside the tile and scatters the values into the term's 256-entry row image
//           in LDS (a dense-value column: one 16-B load per lane of the tile's value bits). Then every wave
//           walks each of its queries' terms in ascending term order and adds fl32(w * v) into
//           that query's fp32 accumulators of the lane's two rows (packed multiply, packed add).
//           Ascending term order per (row, query) is the Qdrant summation order; nothing else
//           is reordered. Per-term cursors carry over to the next tile. Each wave keeps a sorted
//           16-entry list per query (16 lanes each) plus the best score it dropped.
//   merge:  per query, pool the range lists, keep the k best, certify against the dropped
//           bound (scores are exact, so the bound test is strict: k-th > bound).
//   fallback for uncertified queries: the scan rerun in collect mode gathers every row scoring
//           >= the k-th candidate (a lower bound of the true k-th), then sorts them.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <vector>

#include "armi_index.h"

namespace {

constexpr int kQB = 64;                 // queries per pass
constexpr int kQW = 4;                  // queries per wave
constexpr int kWaves = kQB / kQW;       // 16 waves per workgroup
constexpr int kScanThreads = kWaves * 64;
constexpr int kKW = 16;                 // candidates per range and query (16 lanes per query)
constexpr int kSelCap = 1024;           // kept entries per query in the merge
constexpr int kMaxK = 240;
constexpr int kCollectCap = 4096;       // rows per query collected by the fallback
constexpr int kMaxTerms = 256;          // query terms per query (BGE-M3 queries are short)
constexpr int kLongTerm = 256;          // postings from which a term gets a range-start table
constexpr int kPad = 128;               // sentinel slots past the last list (two 64-posting loads)
constexpr int kBatch = 4;  // terms whose LDS reads are in flight together (8: no gain, r04ak)
constexpr int kTile = 256;              // rows per scan step: four adjacent rows per lane
constexpr int kQStride = kMaxTerms + 2 * kBatch;  // list entries per query slot (+ padding)
constexpr int kMaxRanges = 256;
constexpr int kMaxU = kQB * kMaxTerms;  // distinct terms of one pass, at most
constexpr int kU = 64;                  // terms per staging segment
constexpr int kHold = kU / kWaves;      // terms of a segment staged by one wave
constexpr int kRegSegs = 64 / kHold;    // segments whose cursors stay in registers
// segment boundaries 64 .. kMaxU / kU of each query slot (the first 64 stay in registers)
constexpr int kSegTab = kMaxU / kU - 64 + 1;
// two staging buffers, the all-zero row, the 64-entry scratch row of out-of-tile scatters and
// the segment-boundary table (uint16 [kWaves][kQW][kSegTab])
constexpr size_t kScanLdsStage = (size_t)(2 * kU + 1) * kTile * 4 + 64 * 4;
constexpr size_t kScanLds = kScanLdsStage + (size_t)kWaves * kQW * kSegTab * 2;
constexpr size_t kPrepLds = (size_t)kMaxU * 8;         // pass pairs: keys + weights, 128 KB
constexpr int kBitmapVocab = 1 << 18;   // vocabularies up to which a pass numbers its terms by bitmap
constexpr int kBmWords = kBitmapVocab / 32;
constexpr size_t kPrepBmLds = (size_t)kBmWords * 8;    // term bitmap + per-word prefix, 64 KB
constexpr int32_t kEndRow = 0x7fffffff;
constexpr float kNegInf = -std::numeric_limits<float>::infinity();
static_assert(kQW * kKW == 64, "one 16-lane list segment per query of the wave");

// ------------------------------------------------------------------------- index build

__global__ void entry_rows_kernel(const int64_t* __restrict__ indptr, int64_t n_rows,
                                  int32_t* __restrict__ row_of) {
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + armi::wave_id();
  if (r >= n_rows) return;
  for (int64_t e = indptr[r] + (threadIdx.x & 63); e < indptr[r + 1]; e += 64)
    row_of[e] = (int32_t)r;
}

__global__ void count_nonfinite_kernel(const float* __restrict__ values, int64_t nnz,
                                       unsigned long long* __restrict__ bad) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool b = i < nnz && !isfinite(values[i]);
  const unsigned long long m = __ballot(b);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(bad, (unsigned long long)__popcll(m));
}

__global__ void term_keys_kernel(const int32_t* __restrict__ indices, int64_t nnz, int32_t vocab,
                                 uint32_t* __restrict__ keys, int32_t* __restrict__ ent) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nnz) return;
  const int32_t t = indices[i];
  keys[i] = (t >= 0 && t < vocab) ? (uint32_t)t : (uint32_t)vocab;  // invalid ids sort last
  ent[i] = (int32_t)i;
}

// term_ptr[t] = (#entries with term < t) + t: one sentinel slot per preceding term.
__global__ void term_ptr_kernel(const uint32_t* __restrict__ skeys, int64_t nnz, int32_t vocab,
                                int32_t* __restrict__ term_ptr) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > nnz) return;
  const int64_t prev = i == 0 ? -1 : (int64_t)skeys[i - 1];
  const int64_t cur = i == nnz ? (int64_t)vocab : (int64_t)skeys[i];
  for (int64_t t = prev + 1; t <= cur && t <= vocab; ++t) term_ptr[t] = (int32_t)(i + t);
}

__global__ void postings_kernel(const uint32_t* __restrict__ skeys, const int32_t* __restrict__ sent,
                                const int32_t* __restrict__ row_of,
                                const float* __restrict__ values, int64_t nnz, int32_t vocab,
                                int2* __restrict__ post) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nnz) return;
  const uint32_t t = skeys[i];
  if (t >= (uint32_t)vocab) return;
  const int64_t pos = i + t;
  const int32_t e = sent[i];
  // a zero value is kept as -0.0: the scan's staging rows use bit pattern 0 for "no posting",
  // and fl32(w * -0.0) added to an fp32 sum changes it exactly as fl32(w * +0.0) does (not at all)
  const uint32_t v = __float_as_uint(values[e]);
  post[pos] = make_int2(row_of[e], (int32_t)(v == 0u ? 0x80000000u : v));
}

__global__ void sentinels_kernel(const int32_t* __restrict__ term_ptr, int32_t vocab,
                                 int64_t n_postings, int2* __restrict__ post,
                                 int32_t* __restrict__ is_long) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < vocab) {
    const int32_t s = term_ptr[t + 1] - 1;
    post[s] = make_int2(kEndRow, 0);
    is_long[t] = (s - term_ptr[t]) >= kLongTerm ? 1 : 0;
  } else if (t == vocab) {
    is_long[t] = 0;
  }
  if (t < kPad) post[n_postings + t] = make_int2(kEndRow, 0);
}

// dense columns: flag[t] = 1 for a term in >= 1/8 of the rows (df = postings - its sentinel)
__global__ void dense_flag_kernel(const int32_t* __restrict__ term_ptr, int32_t vocab,
                                  int64_t n_rows, int32_t* __restrict__ flag) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < vocab) {
    const int64_t df = term_ptr[t + 1] - 1 - term_ptr[t];
    flag[t] = (df > 0 && df * 8 >= n_rows) ? 1 : 0;
  } else if (t == vocab) {
    flag[t] = 0;
  }
}

__global__ void dense_of_kernel(const int32_t* __restrict__ flag, const int32_t* __restrict__ scan,
                                int32_t vocab, int32_t* __restrict__ dense_of) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < vocab) dense_of[t] = flag[t] ? scan[t] : -1;
}

// value bits of every posting of a dense term into its column (the postings' encoding)
__global__ void dense_fill_kernel(const int32_t* __restrict__ term_ptr,
                                  const int32_t* __restrict__ dense_of,
                                  const int2* __restrict__ post, int64_t n_postings,
                                  const uint32_t* __restrict__ skeys, int64_t nnz, int32_t vocab,
                                  int64_t stride, uint32_t* __restrict__ dense_val) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nnz) return;
  const uint32_t t = skeys[i];
  if (t >= (uint32_t)vocab) return;
  const int32_t d = dense_of[t];
  if (d < 0) return;
  const int2 pv = post[i + t];  // the posting postings_kernel wrote for sorted entry i
  dense_val[(size_t)d * stride + pv.x] = (uint32_t)pv.y;
}

__global__ void long_of_kernel(const int32_t* __restrict__ term_ptr, int32_t vocab,
                               const int32_t* __restrict__ scan, int32_t* __restrict__ long_of) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= vocab) return;
  long_of[t] = (term_ptr[t + 1] - 1 - term_ptr[t]) >= kLongTerm ? scan[t] : -1;
}

// start_tab[l][g] = rank (within term t) of t's first posting with row >= g*R: the posting whose
// (previous row, row] interval holds g*R; the ranges after t's last posting get P_t.
__global__ void start_tab_kernel(const uint32_t* __restrict__ skeys, int64_t nnz, int32_t vocab,
                                 const int32_t* __restrict__ term_ptr,
                                 const int32_t* __restrict__ long_of,
                                 const int2* __restrict__ post, int64_t range_rows,
                                 int n_ranges, int32_t* __restrict__ start_tab) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nnz) return;
  const uint32_t t = skeys[i];
  if (t >= (uint32_t)vocab) return;
  const int32_t l = long_of[t];
  if (l < 0) return;
  const int64_t pos = i + t;
  const int32_t first = term_ptr[t];
  const int32_t last = term_ptr[t + 1] - 2;
  const int32_t rel = (int32_t)(pos - first);
  const int64_t r = post[pos].x;
  const int64_t prev = pos == first ? -1 : (int64_t)post[pos - 1].x;
  int32_t* tab = start_tab + (size_t)l * n_ranges;
  const int64_t g_lo = (prev + range_rows) / range_rows;  // ceil((prev + 1) / R)
  const int64_t g_hi = min(r / range_rows, (int64_t)n_ranges - 1);
  for (int64_t g = g_lo; g <= g_hi; ++g) tab[g] = rel;
  if (pos == last)
    for (int64_t g = r / range_rows + 1; g < n_ranges; ++g) tab[g] = rel + 1;
}

// ------------------------------------------------------------------------- per-pass prep

// One entry of a query's term list: the query's weight and the byte offset of the term's staging
// row within a segment buffer ((u % kU) * kTile * 4). 8 B: a batch of 4 entries is one 32-B scalar
// load, and the weight in the even register of each pair feeds the packed multiply directly.
struct alignas(8) QTerm {
  float w;
  int32_t off;
};

// What a pass_terms block writes for the MFMA filter (sparse_filter.h); fB == nullptr: filter
// off. Per query entry j of slot q's list, fs = the term's u8 scale; per query q (not slot), the
// rescore's term table: fterm = {fp32 column (dense_of) or -1, rare-value table base, its mask,
// the term}, fw = the weight, fnt = the count.
struct FilterPrep {
  const float* term_scale;
  const int32_t* dense_of;
  const int2* rare_of;
  uint16_t* fB;     // the pass's B slices [kFMaxSeg][kQB][kFK] fp16
  float* fscale;    // its key scale
  int32_t* felig;   // [kQB] queries the filter may answer
  float* fs;        // [kQB * kQStride] by slot
  int4* fterm;      // [kQB * kMaxTerms] by query
  float* fw;        // [kQB * kMaxTerms] by query
  int32_t* fnt;     // [kQB] by query
};

// one list entry's filter record (t = its term, w its weight, slot q's entry idx of query qq);
// returns the term's u8 scale
__device__ __forceinline__ float filter_entry(const FilterPrep& fp, int slot, int idx, int qq,
                                              int32_t t, float w) {
  const float s = fp.term_scale[t];
  fp.fs[slot * kQStride + idx] = s;
  const int2 ro = fp.rare_of[t];
  fp.fterm[qq * kMaxTerms + idx] = make_int4(fp.dense_of[t], ro.x, ro.y, t);
  fp.fw[qq * kMaxTerms + idx] = w;
  return s;
}

// a pass_terms wave's lists as the filter prep reads them: per slot i of the wave its query
// (-1: none) and list length, and when the list is one 64-entry chunk (regs), entry j's u,
// weight and scale in lane j
struct PrepCapture {
  int q[kQW];
  int n[kQW];
  bool regs[kQW];
  int u[kQW];
  float w[kQW];
  float s[kQW];
};

// the MFMA filter's per-pass B slices, run at the end of a pass_terms block (sparse_filter.h)
__device__ __forceinline__ void filter_prep_block(int nU, const QTerm* ql, const int32_t* qu,
                                                  const PrepCapture& cap, const FilterPrep& fp);

// Wave 0 of a pass_terms block (tid = lane < 64): per-query term counts (first 256 terms;
// flags[q] = 8 beyond), their exclusive offsets off[0..64], and the query -> slot deal: queries
// sorted by term count (desc, then index) are dealt to the 16 waves in snake order, so each
// wave's sum of term counts (its per-tile work) is about the same; slot 4 w + i of wave w.
__device__ __forceinline__ void deal_queries(const int32_t* __restrict__ q_indptr, int nq, int tid,
                                             int32_t* off, int32_t* qslot,
                                             int32_t* __restrict__ qof,
                                             uint32_t* __restrict__ flags) {
  const int lane = tid;
  int n = 0;
  if (tid < nq) {
    const int32_t len = q_indptr[tid + 1] - q_indptr[tid];
    n = min(len, kMaxTerms);
    flags[tid] = len > kMaxTerms ? 8u : 0u;
  }
  int x = n;  // inclusive scan of the per-query counts
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  off[tid + 1] = x;
  if (tid == 0) off[0] = 0;
  int sk = (tid < nq ? n : -1) * 64 + (63 - tid);
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const int o = armi::xor_stride(sk, stride);
      const bool lower = (lane & stride) == 0;
      const bool desc = (lane & size) == 0;
      if ((lower == desc) ? (o > sk) : (o < sk)) sk = o;
    }
  }
  const int r = lane;  // rank
  const int q = 63 - (sk & 63);
  const int w = ((r >> 4) & 1) ? 15 - (r & 15) : (r & 15);
  const int slot = (w << 2) | (r >> 4);
  qslot[q] = slot;
  qof[slot] = r < nq ? q : -1;
}

// The pass's query terms when vocab <= kBitmapVocab (BGE-M3: 250 002), without a sort: the
// distinct terms are the set bits of an LDS bitmap over the vocabulary, u(t) = the number of set
// bits below t (per-word prefix counts + a popcount), and since every query's indices ascend
// (the C ABI's contract), each slot's list is its query's own terms in CSR order, already in
// ascending u. Same outputs as pass_terms_kernel.
__global__ __launch_bounds__(1024) void pass_terms_bitmap_kernel(
    const int32_t* __restrict__ q_indptr, const int32_t* __restrict__ q_indices,
    const float* __restrict__ q_values, int nq, int32_t vocab, int32_t* __restrict__ uterm,
    int32_t* __restrict__ n_terms, QTerm* __restrict__ ql, int32_t* __restrict__ qu,
    int32_t* __restrict__ qcount, int32_t* __restrict__ qof, uint32_t* __restrict__ flags,
    int32_t* __restrict__ coll_count, FilterPrep fp) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* bits = reinterpret_cast<uint32_t*>(smem);               // [kBmWords]
  int32_t* wpre = reinterpret_cast<int32_t*>(smem + kBmWords * 4);  // [kBmWords]
  __shared__ int32_t off[kQB + 1];
  __shared__ int32_t qslot[kQB];
  __shared__ int32_t wsum[kScanThreads / 64];
  const int tid = threadIdx.x;
  const int wave = armi::wave_id();
  const int lane = tid & 63;
  const int nw = (vocab + 31) >> 5;
  for (int i = tid; i < nw; i += kScanThreads) bits[i] = 0u;
  if (tid < 2 * kQB) coll_count[tid] = 0;  // the pass's collect counters and helper counters
  if (tid < kQB) deal_queries(q_indptr, nq, tid, off, qslot, qof, flags);
  __syncthreads();
  const int total = off[kQB];
  for (int e = tid; e < total; e += kScanThreads) {
    int a = 0, n = kQB;  // q = last index with off[q] <= e
    while (n > 1) {
      const int h = n >> 1;
      if (off[a + h] <= e) a += h;
      n -= h;
    }
    const int32_t t = q_indices[q_indptr[a] + (e - off[a])];
    if (t >= 0 && t < vocab) atomicOr(&bits[t >> 5], 1u << (t & 31));
  }
  __syncthreads();
  // exclusive prefix of the per-word set-bit counts (kPer consecutive words per thread), and
  // uterm[u] = t for every set bit
  constexpr int kPer = kBmWords / kScanThreads;
  int cnt[kPer];
  int sum = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int w = tid * kPer + j;
    cnt[j] = w < nw ? __popc(bits[w]) : 0;
    sum += cnt[j];
  }
  int x = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  int run = x - sum;
  for (int v = 0; v < wave; ++v) run += wsum[v];
  if (tid == kScanThreads - 1) *n_terms = run + sum;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int w = tid * kPer + j;
    if (w < nw) {
      wpre[w] = run;
      uint32_t b = bits[w];
      int u = run;
      while (b) {
        uterm[u++] = w * 32 + __builtin_ctz(b);
        b &= b - 1u;
      }
    }
    run += cnt[j];
  }
  __syncthreads();
  // wave w writes the lists of slots 4 w + i
  PrepCapture cap;
#pragma unroll
  for (int i = 0; i < kQW; ++i) {
    const int slot = wave * kQW + i;
    const int q = qof[slot];
    int m = 0;
    cap.u[i] = 0;
    cap.w[i] = 0.f;
    cap.s[i] = 0.f;
    bool full = true;  // every term of the query valid (then entry j of the list = term j)
    int n = 0;
    if (q >= 0) {
      const int32_t p0 = q_indptr[q];
      n = off[q + 1] - off[q];
      for (int c0 = 0; c0 < n; c0 += 64) {
        const int j = c0 + lane;
        const int32_t t = j < n ? q_indices[p0 + j] : -1;
        const bool ok = t >= 0 && t < vocab;
        const unsigned long long mb = __ballot(ok);
        full &= __popcll(mb) == min(64, n - c0);
        if (ok) {
          const int idx = m + __popcll(mb & ((1ull << lane) - 1ull));
          const int32_t u = wpre[t >> 5] + __popc(bits[t >> 5] & ((1u << (t & 31)) - 1u));
          const float w = q_values[p0 + j];
          ql[slot * kQStride + idx] = QTerm{w, (u % kU) * kTile * 4};
          qu[slot * kQStride + idx] = u;
          if (fp.fB && idx < kMaxTerms) {
            const float s = filter_entry(fp, slot, idx, q, t, w);
            if (c0 == 0) {
              cap.u[i] = u;
              cap.w[i] = w;
              cap.s[i] = s;
            }
          }
        }
        m += __popcll(mb);
      }
    }
    cap.q[i] = q;
    cap.n[i] = m;
    cap.regs[i] = full && n <= 64;
    // a batch of the scan may read up to kBatch - 1 entries past a list: finite weights there
    if (lane < kBatch) ql[slot * kQStride + m + lane] = QTerm{0.f, 0};
    if (lane == 0) qcount[slot] = m;
    if (fp.fB && lane == 0 && q >= 0) fp.fnt[q] = m;
  }
  if (fp.fB) {  // uniform: the MFMA filter runs on this pass
    __syncthreads();
    int nU = 0;
    for (int v = 0; v < kScanThreads / 64; ++v) nU += wsum[v];
    filter_prep_block(nU, ql, qu, cap, fp);
  }
}

// One block for the pass. Sorts the pass's (term, query) pairs by (term, slot) where query q sits
// in slot 4 w + i of wave w, numbers the distinct terms u = 0..nU-1 ascending (uterm[u] = term),
// and builds per slot the ascending list of its query's terms: (staging offset, weight) in ql and
// u in qu, qcount entries.
// flags[q] = 8 when a query has more than 256 terms (the first 256 are used).
__global__ __launch_bounds__(1024) void pass_terms_kernel(
    const int32_t* __restrict__ q_indptr, const int32_t* __restrict__ q_indices,
    const float* __restrict__ q_values, int nq, int32_t vocab, int32_t* __restrict__ uterm,
    int32_t* __restrict__ n_terms, QTerm* __restrict__ ql, int32_t* __restrict__ qu,
    int32_t* __restrict__ qcount, int32_t* __restrict__ qof, uint32_t* __restrict__ flags,
    int32_t* __restrict__ coll_count, FilterPrep fp) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* key = reinterpret_cast<uint32_t*>(smem);           // [kMaxU]
  float* val = reinterpret_cast<float*>(smem + kMaxU * 4);     // [kMaxU]
  __shared__ int32_t off[kQB + 1];
  __shared__ int32_t qslot[kQB];
  __shared__ int32_t part[1024];
  const int tid = threadIdx.x;
  const int wave = armi::wave_id();
  const int lane = tid & 63;
  if (tid < 2 * kQB) coll_count[tid] = 0;  // the pass's collect counters and helper counters
  if (tid < kQB) deal_queries(q_indptr, nq, tid, off, qslot, qof, flags);
  __syncthreads();
  const int total = off[kQB];
  const int n2 = armi::pow2_at_least(max(total, 2));
  for (int e = tid; e < n2; e += 1024) {
    uint32_t k = 0xffffffffu;
    float v = 0.f;
    if (e < total) {
      int a = 0, n = kQB;  // q = last index with off[q] <= e
      while (n > 1) {
        const int h = n >> 1;
        if (off[a + h] <= e) a += h;
        n -= h;
      }
      const int q = a;
      const int32_t p = q_indptr[q] + (e - off[q]);
      const int32_t t = q_indices[p];
      if (t >= 0 && t < vocab) {
        k = ((uint32_t)t << 6) | (uint32_t)qslot[q];
        v = q_values[p];
      }
    }
    key[e] = k;
    val[e] = v;
  }
  if (n2 <= 1024) {
    // one element per thread: in-wave stages by shuffles, cross-wave stages through LDS
    __syncthreads();
    uint32_t kk = tid < n2 ? key[tid] : 0xffffffffu;
    float vv = tid < n2 ? val[tid] : 0.f;
    for (int size = 2; size <= n2; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        uint32_t ok;
        float ov;
        if (stride >= 64) {
          __syncthreads();
          key[tid] = kk;
          val[tid] = vv;
          __syncthreads();
          ok = key[tid ^ stride];
          ov = val[tid ^ stride];
        } else {
          ok = (uint32_t)__shfl_xor((int)kk, stride);
          ov = __shfl_xor(vv, stride);
        }
        const bool lower = (tid & stride) == 0;
        const bool up = (tid & size) == 0;
        if ((lower == up) ? (ok < kk) : (ok > kk)) {
          kk = ok;
          vv = ov;
        }
      }
    }
    __syncthreads();
    if (tid < n2) {
      key[tid] = kk;
      val[tid] = vv;
    }
  } else {
    for (int size = 2; size <= n2; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        __syncthreads();
        for (int e = tid; e < n2; e += 1024) {
          const int o = e ^ stride;
          if (o > e) {
            const bool up = (e & size) == 0;
            const uint32_t x = key[e], y = key[o];
            if ((x > y) == up) {
              key[e] = y;
              key[o] = x;
              const float tv = val[e];
              val[e] = val[o];
              val[o] = tv;
            }
          }
        }
      }
    }
  }
  __syncthreads();
  // u = rank of the distinct term: per-thread head counts over consecutive slots, then a scan
  const int per = (n2 + 1023) / 1024;
  const int e0 = tid * per, e1 = min(n2, e0 + per);
  int heads = 0;
  for (int e = e0; e < e1; ++e)
    heads += (key[e] != 0xffffffffu && (e == 0 || (key[e] >> 6) != (key[e - 1] >> 6))) ? 1 : 0;
  part[tid] = heads;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const int x = tid >= d ? part[tid - d] : 0;
    __syncthreads();
    part[tid] += x;
    __syncthreads();
  }
  int u = part[tid] - heads - 1;
  uint32_t rek[16];  // per <= 16 (n2 <= 16384)
  for (int e = e0; e < e1; ++e) {
    const uint32_t k = key[e];
    if (k != 0xffffffffu && (e == 0 || (k >> 6) != (key[e - 1] >> 6))) {
      ++u;
      uterm[u] = (int32_t)(k >> 6);
    }
    rek[e - e0] = k == 0xffffffffu ? k : (((uint32_t)u << 6) | (k & 63u));
  }
  if (tid == 1023) *n_terms = part[1023];
  __syncthreads();
  for (int e = e0; e < e1; ++e) key[e] = rek[e - e0];  // term id -> u (same order)
  __syncthreads();
  // wave w of this block writes the lists of slots 4 w + i: its queries' terms, ascending u
  int run[kQW] = {0, 0, 0, 0};
  for (int c0 = 0; c0 < n2; c0 += 64) {
    const int e = c0 + lane;
    const uint32_t k = e < n2 ? key[e] : 0xffffffffu;  // LDS past n2 was never written
#pragma unroll
    for (int i = 0; i < kQW; ++i) {
      const int slot = wave * kQW + i;
      const bool mine = k != 0xffffffffu && (int)(k & 63u) == slot;
      const unsigned long long mb = __ballot(mine);
      if (mine) {
        const int idx = run[i] + __popcll(mb & ((1ull << lane) - 1ull));
        const int32_t u = (int32_t)(k >> 6);
        ql[slot * kQStride + idx] = QTerm{val[e], (u % kU) * kTile * 4};
        qu[slot * kQStride + idx] = u;
        if (fp.fB) filter_entry(fp, slot, idx, qof[slot], uterm[u], val[e]);
      }
      run[i] += __popcll(mb);
    }
  }
  // a batch of the scan may read up to kBatch - 1 entries past a list: finite weights there
#pragma unroll
  for (int i = 0; i < kQW; ++i)
    if (lane < kBatch) ql[(wave * kQW + i) * kQStride + run[i] + lane] = QTerm{0.f, 0};
  if (lane < kQW) {
    const int c = lane == 0 ? run[0] : lane == 1 ? run[1] : lane == 2 ? run[2] : run[3];
    qcount[wave * kQW + lane] = c;
    const int q = qof[wave * kQW + lane];
    if (fp.fB && q >= 0) fp.fnt[q] = c;
  }
  if (fp.fB) {  // uniform: the MFMA filter runs on this pass (lists read back from memory)
    __syncthreads();
    PrepCapture cap;
#pragma unroll
    for (int i = 0; i < kQW; ++i) {
      const int slot = wave * kQW + i;
      cap.q[i] = qof[slot];
      cap.n[i] = run[i];
      cap.regs[i] = false;
    }
    filter_prep_block(part[1023], ql, qu, cap, fp);
  }
}

// ------------------------------------------------------------------------- scan

#ifdef ARMI_SPARSE_PROFILE
// Profiling build only (ARMI_BUILD_FLAGS=-DARMI_SPARSE_PROFILE): per-wave phase timers and the
// ARMI_SPARSE_DBG knobs (1 = skip compute, 2 = stage nothing, 4 = no step barrier, 8 = report,
// 16 = clear every staged row each step).
// 12 words per wave: 6 phase sums, term count, steps, setup, tail, entry and exit stamps
__device__ unsigned long long g_sparse_prof[kMaxRanges * kWaves * 12];
#define ARMI_PROF_T(x) x = wall_clock64()
#define ARMI_PROF_ADD(i, a, b) tp[i] += (b) - (a)
#else
#define ARMI_PROF_T(x) (void)0
#define ARMI_PROF_ADD(i, a, b) (void)0
#endif

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int rl_i(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ float rl_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

__device__ __forceinline__ uint32_t or3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_or3_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// first posting of term t at or after row `lo` (range g), with its row
__device__ __forceinline__ int2 range_cursor(int32_t t, int g, int64_t lo, int n_ranges,
                                             const int32_t* __restrict__ term_ptr,
                                             const int32_t* __restrict__ long_of,
                                             const int32_t* __restrict__ start_tab,
                                             const int2* __restrict__ post) {
  const int32_t b = term_ptr[t];
  const int32_t l = long_of[t];
  int32_t c;
  if (l >= 0) {
    c = b + start_tab[(size_t)l * n_ranges + g];
  } else {
    int32_t a = b, n = term_ptr[t + 1] - 1 - b;
    while (n > 0) {
      const int32_t h = n >> 1;
      if (post[a + h].x < lo) {
        a += h + 1;
        n -= h + 1;
      } else {
        n = h;
      }
    }
    c = a;
  }
  return make_int2(c, post[c].x);
}

// Workgroup = one row range; steps = (256-row tile, segment of kU = 64 pass terms). Staging: term
// u_local of the segment is held by wave u_local & 15 (lane slot u_local >> 4), which keeps its
// cursor, loads the term's next 128 postings (lane-reversed: postings c + 2 (63 - l) and + 1 in
// lane l; a further 128 at a time while all of them fall inside the tile), keeps the prefix inside
// the tile and scatters the value bits to buf[u_local][row - tile start] in LDS (0 = no posting).
// Compute: lane l owns rows 4l .. 4l + 3 of the tile; wave w walks each of its 4 queries' terms of
// the segment in ascending u, reads the four rows buf[u_local][4l .. 4l + 3] (one ds_read_b128)
// and adds fl32(w * v) into the query's four fp32 accumulators (two packed multiplies, two packed
// adds). Round 5: 256-row tiles of 64-term segments (was 128 rows x 128 terms, two rows per
// lane): the per-term list entry, address add and LDS read serve four rows instead of two. Staging of step s+1 is issued
// before, and written after, the compute of step s (double-buffered LDS, one barrier per step).
// kCollect = false: per-range candidate lists; kCollect = true: every row scoring >= thr.
template <bool kCollect>
__global__ __launch_bounds__(kScanThreads) void sparse_scan_kernel(
    const int32_t* __restrict__ term_ptr, const int2* __restrict__ post,
    const int32_t* __restrict__ long_of,
    const int32_t* __restrict__ start_tab, int64_t n_rows, int64_t range_rows, int n_ranges,
    const uint64_t* __restrict__ row_mask, int nq, const int32_t* __restrict__ uterm,
    const int32_t* __restrict__ n_terms, const QTerm* __restrict__ ql,
    const int32_t* __restrict__ qu, const int32_t* __restrict__ qcount,
    const int32_t* __restrict__ qof, int2* __restrict__ cursors,
    float* __restrict__ cand_key, int32_t* __restrict__ cand_row, float* __restrict__ cand_bound,
    const float* __restrict__ thr, int* __restrict__ coll_count, float* __restrict__ coll_key,
    int32_t* __restrict__ coll_row, int dbg, const int32_t* __restrict__ dense_of,
    const uint32_t* __restrict__ dense_val, int64_t dense_stride,
    const uint32_t* __restrict__ done_flags) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sbuf[];  // [2][kU][kTile]
#ifdef ARMI_SPARSE_PROFILE
  const unsigned long long t_entry = wall_clock64();
#endif
  const int g = blockIdx.x;
  const int wave = armi::wave_id();
  const int lane = threadIdx.x & 63;
  int qw[kQW];  // this wave's queries (-1: none)
#pragma unroll
  for (int i = 0; i < kQW; ++i) qw[i] = qof[wave * kQW + i];
  if constexpr (!kCollect) {
    // queries the MFMA filter already answered (done_flags: the pass's flags) are dropped; with
    // none left the whole grid exits here (the flags are the same for every workgroup)
    if (done_flags) {
      bool any = false;
#pragma unroll
      for (int i = 0; i < kQW; ++i) {
        if (qw[i] >= 0 && (done_flags[qw[i]] & ARMI_FLAG_CERTIFIED)) qw[i] = -1;
        any |= qw[i] >= 0;
      }
      if (!__syncthreads_or(any)) return;  // workgroup-uniform
    }
  }
  const bool has_q = qw[0] >= 0 || qw[1] >= 0 || qw[2] >= 0 || qw[3] >= 0;
  float tq[kQW];
  if constexpr (kCollect) {
    bool any = false;
#pragma unroll
    for (int i = 0; i < kQW; ++i) {
      const int q = qw[i];
      tq[i] = q >= 0 ? thr[q] : std::numeric_limits<float>::infinity();
      any |= tq[i] != std::numeric_limits<float>::infinity();
    }
    if (!__syncthreads_or(any)) return;  // workgroup-uniform
  }
  const int nU = *n_terms;
  const int nSeg = (nU + kU - 1) / kU;
  const int64_t lo = (int64_t)g * range_rows;
  const int64_t hi = min(lo + range_rows, n_rows);
  const int n_tiles = hi > lo ? (int)((hi - lo + kTile - 1) / kTile) : 0;
  int2* gcur = cursors + (size_t)g * kMaxU;

  // cursors of the held terms: segments < kRegSegs in lane 8*seg + slot, the rest in memory
  int2 creg = make_int2(0, kEndRow);
  {
    const int s = lane / kHold, u = s * kU + (lane % kHold) * kWaves + wave;
    if (s < nSeg && u < nU) {
      const int32_t t = uterm[u];
      const int32_t d = dense_of[t];
      creg = d >= 0 ? make_int2(-(d + 1), 0)
                    : range_cursor(t, g, lo, n_ranges, term_ptr, long_of, start_tab, post);
    }
  }
  for (int s = kRegSegs; s < nSeg; ++s) {
    const int u = s * kU + lane * kWaves + wave;
    if (lane < kHold && u < nU) {
      const int32_t t = uterm[u];
      const int32_t d = dense_of[t];
      gcur[u] = d >= 0 ? make_int2(-(d + 1), 0)
                       : range_cursor(t, g, lo, n_ranges, term_ptr, long_of, start_tab, post);
    }
  }

  // per lane (= row pair within the tile) and query: the two best rows seen in this lane, plus
  // the best score dropped from the lane
  float l1s[kQW], l2s[kQW], disc[kQW];
  int32_t l1r[kQW], l2r[kQW];
#pragma unroll
  for (int i = 0; i < kQW; ++i) {
    l1s[i] = kNegInf;
    l2s[i] = kNegInf;
    disc[i] = kNegInf;
    l1r[i] = kEndRow;
    l2r[i] = kEndRow;
  }
  f2 acc[kQW], acc2[kQW];  // rows 4 lane, + 1 (acc) and + 2, + 3 (acc2)
  uint32_t hm[kQW][4];  // per row: OR of the staged value bits seen, != 0 <=> a shared term
#pragma unroll
  for (int i = 0; i < kQW; ++i) {
    acc[i] = f2{0.f, 0.f};
    acc2[i] = f2{0.f, 0.f};
#pragma unroll
    for (int h = 0; h < 4; ++h) hm[i][h] = 0u;
  }

  // staged postings of the held terms: lane l holds postings c + 2 (63 - l) (.x row, .y value
  // bits) and c + 2 (63 - l) + 1 (.z, .w) of the term's cursor c: one 16-B load per term
  typedef int32_t p4 __attribute__((ext_vector_type(4), aligned(8)));
  p4 sp[kHold];
  uint32_t amask = 0;
  uint32_t dmask = 0;  // held terms of the staged step that are dense columns (cursor.x < 0)
  int2 scv = make_int2(0, kEndRow);
  const int rev2 = 2 * (63 - lane);
  // scatter target of a lane whose posting is outside the tile: a 64-entry scratch row
  uint32_t* const trash = sbuf + (size_t)(2 * kU + 1) * kTile + lane;
  auto tile_hi = [&](int tile) { return (int32_t)min(lo + (int64_t)(tile + 1) * kTile, hi); };
  auto issue = [&](int tile, int seg) {
    const int32_t thi = tile_hi(tile);
    const int base = seg < kRegSegs ? seg * kHold : 0;
    int2 cv = creg;
    const int l = lane - base;
    const int u = seg * kU + l * kWaves + wave;
    const bool mine = l >= 0 && l < kHold && u < nU;
    if (seg >= kRegSegs) cv = mine ? gcur[u] : make_int2(0, kEndRow);
    amask = (uint32_t)(__ballot(mine && cv.y < thi) >> base) & ((1u << kHold) - 1u);
    dmask = (uint32_t)(__ballot(mine && cv.x < 0) >> base) & ((1u << kHold) - 1u);
    if (dbg & 2) amask = 0;
    scv = cv;
    const int64_t tlo = lo + (int64_t)tile * kTile;
#pragma unroll
    for (int k = 0; k < kHold; ++k) {
      if ((amask >> k) & 1u) {
        const int cx = rl_i(cv.x, base + k);  // uniform
        if (cx < 0) {
          // dense column: the tile's value bits, rows tlo + 4 lane .. + 3 (zero past the store):
          // one whole 16-B load per lane
          sp[k] = *reinterpret_cast<const p4*>(dense_val + (size_t)(-cx - 1) * dense_stride + tlo +
                                               4 * lane);
        } else {
          sp[k] = *reinterpret_cast<const p4*>(post + cx + rev2);
        }
      }
    }
  };
  // Every held row image is cleared, then the postings inside the tile are scattered into it
  // (lanes whose posting lies outside write the scratch row instead: no exec-mask branches).
  // The in-tile postings are a prefix of the 128 loaded (rows ascend to the list's sentinel):
  // with ne / no the even / odd positions' in-tile prefixes (lane 63 holds positions 0 and 1),
  // the prefix length is min(2 ne, 2 no + 1).
  // rows of this wave's held terms per staging buffer that hold postings from their last use
  // (round 3: only those are cleared; a row whose term had no posting in its tile is still
  // all-zero, and with Zipf query terms about half the (tile, term) pairs are empty, so this
  // halves the clearing stores, the scan's largest LDS-store item). LDS starts undefined: all dirty.
  uint32_t dirty[2] = {(1u << kHold) - 1u, (1u << kHold) - 1u};
  auto finish = [&](int tile, int seg, int par) {
    const int32_t tlo = (int32_t)(lo + (int64_t)tile * kTile);
    const int32_t thi = tile_hi(tile);
    const int base = seg < kRegSegs ? seg * kHold : 0;
    uint32_t* buf = sbuf + (size_t)par * kU * kTile;
    const uint32_t dm = (dbg & 16) ? (1u << kHold) - 1u : dirty[par];
    dirty[par] = amask;
#pragma unroll
    for (int k = 0; k < kHold; ++k) {
      uint32_t* row = buf + (k * kWaves + wave) * kTile;
      if ((amask & dmask) >> k & 1u) {  // dense column: the whole row image, no clear, no cursor
        reinterpret_cast<p4*>(row)[lane] = sp[k];
        continue;
      }
      if ((dm >> k) & 1u) reinterpret_cast<p4*>(row)[lane] = p4{0, 0, 0, 0};
      if ((amask >> k) & 1u) {
        // a 256-row tile can hold more than the 128 postings of one load: the rest are loaded
        // here, 128 at a time (rare for a term in < 1/8 of the rows), until the list leaves the
        // tile
        p4 v = sp[k];
        int adv = 0;  // postings consumed before v
        while (true) {  // wave-uniform trip count
          const uint64_t be = __ballot(v.x < thi), bo = __ballot(v.z < thi);
          const int ne = be == ~0ull ? 64 : __builtin_clzll(~be);
          const int no = bo == ~0ull ? 64 : __builtin_clzll(~bo);
          const int n = min(2 * ne, 2 * no + 1);  // postings of v inside the tile
          // values are stored with 0.0 as -0.0 (index build), so a posting is never the 0 marker
          uint32_t* d0 = rev2 < n ? row + (v.x - tlo) : trash;
          uint32_t* d1 = rev2 + 1 < n ? row + (v.z - tlo) : trash;
          *d0 = (uint32_t)v.y;
          *d1 = (uint32_t)v.w;
          if (n < 128) {
            // the next posting's row (lane 63 - n / 2 holds positions n & ~1 and n | 1)
            const int nl = 63 - (n >> 1);
            const int32_t re = rl_i(v.x, nl), ro = rl_i(v.z, nl);
            const bool me = lane == base + k;
            scv.x = me ? scv.x + adv + n : scv.x;
            scv.y = me ? ((n & 1) ? ro : re) : scv.y;
            break;
          }
          adv += 128;
          const int cx = rl_i(scv.x, base + k) + adv;  // uniform
          v = *reinterpret_cast<const p4*>(post + cx + rev2);
        }
      }
    }
    if (seg < kRegSegs) {
      creg = scv;
    } else {
      const int u = seg * kU + lane * kWaves + wave;
      if (lane < kHold && u < nU) gcur[u] = scv;
    }
  };
  // qf[i] (lane s): first entry of query slot i's list whose term lies in segment s or later;
  // segments 64 .. kMaxU / kU in the LDS table segtab (a pass has at most 256 segments)
  uint16_t* const segtab = reinterpret_cast<uint16_t*>(reinterpret_cast<unsigned char*>(sbuf) +
                                                       kScanLdsStage) +
                           (size_t)wave * kQW * kSegTab;
  int qn[kQW], qf[kQW];
#pragma unroll
  for (int i = 0; i < kQW; ++i) {
    const int slot = wave * kQW + i;
    qn[i] = qw[i] >= 0 ? qcount[slot] : 0;
    const int32_t* U = qu + slot * kQStride;
    auto lower_seg = [&](int sg) {
      int a0 = 0, n = qn[i];
      while (n > 0) {
        const int h = n >> 1;
        if (U[a0 + h] < sg * kU) {
          a0 += h + 1;
          n -= h + 1;
        } else {
          n = h;
        }
      }
      return a0;
    };
    qf[i] = lane <= nSeg ? lower_seg(lane) : qn[i];
    for (int sg = 64 + lane; sg < nSeg; sg += 64)  // (only waves' own entries: no barrier needed)
      segtab[i * kSegTab + sg - 64] = (uint16_t)lower_seg(sg);
  }
  auto first_of = [&](int i, int sg) {  // sg is wave-uniform
    return sg >= nSeg ? qn[i]
                      : (sg < 64 ? rl_i(qf[i], sg)
                                 : __builtin_amdgcn_readfirstlane((int)segtab[i * kSegTab + sg - 64]));
  };
  auto compute = [&](int seg, int par) {
    const char* buf = reinterpret_cast<const char*>(sbuf + (size_t)par * kU * kTile) + lane * 16;
    const int zoff = (2 - par) * kU * kTile * 4;  // the all-zero row, relative to buf
    // staged rows hold the posting's value bits (a zero value as -0.0), 0 = no posting; a row
    // without a posting adds fl32(w * 0) = +-0, which leaves an fp32 sum unchanged. Batches of
    // 4 entries; entries past the segment's end (the next segment's, or the zero padding after
    // the list: finite weights) read the all-zero row, so they add +-0 as well.
    auto math = [&](const QTerm* tm, const uint4* rv, int i) {
#pragma unroll
      for (int k = 0; k < kBatch; ++k) {
        acc[i] = acc[i] + f2{tm[k].w, tm[k].w} * f2{__uint_as_float(rv[k].x), __uint_as_float(rv[k].y)};
        acc2[i] = acc2[i] + f2{tm[k].w, tm[k].w} * f2{__uint_as_float(rv[k].z), __uint_as_float(rv[k].w)};
      }
#pragma unroll
      for (int k = 0; k < kBatch; k += 2) {
        hm[i][0] = or3(hm[i][0], rv[k].x, rv[k + 1].x);
        hm[i][1] = or3(hm[i][1], rv[k].y, rv[k + 1].y);
        hm[i][2] = or3(hm[i][2], rv[k].z, rv[k + 1].z);
        hm[i][3] = or3(hm[i][3], rv[k].w, rv[k + 1].w);
      }
    };
    auto batch = [&](const QTerm* tm, int tail, int i) {
      uint4 rv[kBatch];
#pragma unroll
      for (int k = 0; k < kBatch; ++k)
        rv[k] = *reinterpret_cast<const uint4*>(buf + (k < tail ? tm[k].off : zoff));
      math(tm, rv, i);
    };
    // The next batch's entries (one scalar load) are requested right after this batch's LDS
    // reads, so the two latencies overlap: the loop waits once per batch for both (scalar loads
    // complete out of order, so any wait on one is a wait on every outstanding LDS read too).
    // Round 3 loaded each batch's entries after the previous batch's math: a scalar-load and an
    // LDS round trip in series per 4 terms (SQ counters r04d: the compute phase latency-bound).
    // Prefetching past a list reads the zero padding or the next slot's entries (inside ql:
    // kQStride = kMaxTerms + 2 kBatch), never used.
#pragma unroll
    for (int i = 0; i < kQW; ++i) {
      const QTerm* L = ql + (wave * kQW + i) * kQStride;
      const int j1 = first_of(i, seg + 1);
      int j = first_of(i, seg);
      if (j >= j1) continue;  // uniform
      QTerm cur[kBatch];
#pragma unroll
      for (int k = 0; k < kBatch; ++k) cur[k] = L[j + k];  // uniform: one scalar load
      for (; j + kBatch <= j1; j += kBatch) {
        QTerm nxt[kBatch];  // requested first: in flight with this batch's LDS reads
#pragma unroll
        for (int k = 0; k < kBatch; ++k) nxt[k] = L[j + kBatch + k];
        uint4 rv[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; ++k) rv[k] = *reinterpret_cast<const uint4*>(buf + cur[k].off);
        math(cur, rv, i);
#pragma unroll
        for (int k = 0; k < kBatch; ++k) cur[k] = nxt[k];
      }
      if (j < j1) batch(cur, j1 - j, i);  // cur = entries j .. j + 3
    }
  };
  auto candidates = [&](int tile, uint64_t mw) {
    const int32_t tlo = (int32_t)(lo + (int64_t)tile * kTile);
    const int32_t thi = tile_hi(tile);
    const int32_t r0 = tlo + 4 * lane;
    const uint32_t mb = (uint32_t)(mw >> ((4 * lane) & 63)) & 0xfu;  // the lane's four rows
#pragma unroll
    for (int i = 0; i < kQW; ++i) {
#pragma unroll
      for (int h = 0; h < 4; ++h) {  // the lane's four rows, ascending
        const bool cand = ((mb >> h) & 1u) && r0 + h < thi && hm[i][h] != 0u;
        const float sc = h == 0 ? acc[i].x : h == 1 ? acc[i].y : h == 2 ? acc2[i].x : acc2[i].y;
        const int32_t r = r0 + h;
        if constexpr (kCollect) {
          const int q = qw[i];
          if (cand && sc >= tq[i]) {
            const int slot = atomicAdd(&coll_count[q], 1);
            if (slot < kCollectCap) {
              coll_key[(size_t)q * kCollectCap + slot] = sc;
              coll_row[(size_t)q * kCollectCap + slot] = r;
            }
          }
        } else {
          // rows reach a lane in ascending order, so strict > keeps equal keys in row order
          const float x = cand ? sc : kNegInf;
          const bool c1 = x > l1s[i];
          const bool c2 = x > l2s[i];
          disc[i] = fmaxf(disc[i], c2 ? l2s[i] : x);
          l2s[i] = c1 ? l1s[i] : (c2 ? x : l2s[i]);
          l2r[i] = c1 ? l1r[i] : (c2 ? r : l2r[i]);
          l1s[i] = c1 ? x : l1s[i];
          l1r[i] = c1 ? r : l1r[i];
        }
      }
    }
  };

  // the all-zero row after the two staging buffers (read by the padding entries of a batch)
  if (threadIdx.x < kTile / 4)
    reinterpret_cast<uint4*>(sbuf + (size_t)2 * kU * kTile)[threadIdx.x] = make_uint4(0u, 0u, 0u, 0u);
  const int S = n_tiles * nSeg;
  unsigned long long tp[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long t_a = 0, t_b = 0;
  (void)tp;
  (void)t_a;
  (void)t_b;
  ARMI_PROF_T(t_a);
#ifdef ARMI_SPARSE_PROFILE
  const unsigned long long t_setup = t_a - t_entry;
#endif
  if (S > 0) {
    issue(0, 0);
    finish(0, 0, 0);
  }
  __syncthreads();
  ARMI_PROF_T(t_b);
  ARMI_PROF_ADD(5, t_a, t_b);
  int tile = 0, seg = 0;  // of step s
  for (int s = 0; s < S; ++s) {
    const int par = s & 1;
    const bool last_seg = seg == nSeg - 1;
    const int tile1 = last_seg ? tile + 1 : tile, seg1 = last_seg ? 0 : seg + 1;  // step s + 1
    // loaded now, used after this step's compute; lo is a multiple of 64, so the lane's four
    // rows tlo + 4 lane .. + 3 are bits of word tlo / 64 + lane / 16
    uint64_t mw = ~0ull;
    if (row_mask && last_seg) {
      const int64_t tlo = lo + (int64_t)tile * kTile;
      const int64_t w0 = tlo + 64 * (lane >> 4);
      mw = w0 < hi ? row_mask[w0 >> 6] : 0ull;
    }
    ARMI_PROF_T(t_a);
    if (s + 1 < S) issue(tile1, seg1);
    ARMI_PROF_T(t_b);
    ARMI_PROF_ADD(0, t_a, t_b);
    if (has_q) {
      if (seg == 0) {
#pragma unroll
        for (int i = 0; i < kQW; ++i) {
          acc[i] = f2{0.f, 0.f};
          acc2[i] = f2{0.f, 0.f};
#pragma unroll
          for (int h = 0; h < 4; ++h) hm[i][h] = 0u;
        }
      }
      if (!(dbg & 1)) compute(seg, par);
      ARMI_PROF_T(t_a);
      ARMI_PROF_ADD(1, t_b, t_a);
      if (last_seg) candidates(tile, mw);
      ARMI_PROF_T(t_b);
      ARMI_PROF_ADD(2, t_a, t_b);
    }
    if (s + 1 < S) finish(tile1, seg1, par ^ 1);
    ARMI_PROF_T(t_a);
    ARMI_PROF_ADD(3, t_b, t_a);
    if (!(dbg & 4)) __syncthreads();
    ARMI_PROF_T(t_b);
    ARMI_PROF_ADD(4, t_a, t_b);
    tile = tile1;
    seg = seg1;
  }
#ifdef ARMI_SPARSE_PROFILE
  const unsigned long long t_loop_end = wall_clock64();
#endif
  if constexpr (!kCollect) {
    if (has_q) {
      // per query: top 16 of the 128 lane entries. Sorting the lanes' best entries (l1) leaves
      // the 16 best in lanes 0 .. 15; a second entry (l2) ranks below its own lane's l1, so only
      // the l2 of those 16 lanes can reach the top 16: lanes 16 .. 31 take them (the lane that
      // owns a row r is ((r - lo) mod kTile) / 4), and one more sort of those 32 gives the top 16.
      // The bound is the 17th best key: max(the 17th l1, the 17th of the 32) (round 5; was two
      // full sorts of l1 and l2, a bitonic split of their heads and a third sort).
      float ka[kQW], ck[kQW], bq[kQW];
      int32_t ra[kQW], cr[kQW];
#pragma unroll
      for (int i = 0; i < kQW; ++i) {
        ka[i] = l1s[i];
        ra[i] = l1r[i];
      }
      armi::wave_sort_approx_desc_n<kQW>(ka, ra);
      const int e = lane & 15;
#pragma unroll
      for (int i = 0; i < kQW; ++i) {
        const float ke = __shfl(ka[i], e);
        const int32_t re = __shfl(ra[i], e);
        const int src = ke == kNegInf ? 0 : (int)(((int64_t)re - lo) & (kTile - 1)) >> 2;
        const float pk = __shfl(l2s[i], src);
        const int32_t pr = __shfl(l2r[i], src);
        const bool part = lane >= 16 && lane < 32 && ke != kNegInf;
        ck[i] = lane < 16 ? ka[i] : (part ? pk : kNegInf);
        cr[i] = lane < 16 ? ra[i] : (part ? pr : kEndRow);
        const float lose16 = __shfl(ka[i], 16);
        bq[i] = fmaxf(disc[i], lane == 0 ? lose16 : kNegInf);
      }
      armi::wave_sort_approx_desc_n<kQW>(ck, cr);
#pragma unroll
      for (int i = 0; i < kQW; ++i) {
        const float lose2 = __shfl(ck[i], 16);
        bq[i] = fmaxf(bq[i], lane == 0 ? lose2 : kNegInf);
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int i = 0; i < kQW; ++i) bq[i] = fmaxf(bq[i], armi::xor_stride(bq[i], o));
#pragma unroll
      for (int i = 0; i < kQW; ++i) {
        const int q = qw[i];
        if (q >= 0) {
          const size_t base = (size_t)g * kQB + q;
          if (lane < kKW) {
            cand_key[base * kKW + lane] = ck[i];
            cand_row[base * kKW + lane] = cr[i];
          }
          if (lane == 0) cand_bound[base] = bq[i];
        }
      }
    }
  }
#ifdef ARMI_SPARSE_PROFILE
  if ((dbg & 8) && lane == 0) {
    const unsigned long long t_exit = wall_clock64();
    unsigned long long* pr = g_sparse_prof + ((size_t)g * kWaves + wave) * 12;
#pragma unroll
    for (int i = 0; i < 6; ++i) pr[i] = tp[i];
    pr[6] = qn[0] + qn[1] + qn[2] + qn[3];
    pr[7] = S;
    pr[8] = t_setup;
    pr[9] = t_exit - t_loop_end;
    pr[10] = t_entry;
    pr[11] = t_exit;
  }
#endif
}

// Order-preserving map of a float to uint32 (larger float -> larger key; -inf lowest).
__device__ __forceinline__ uint32_t ord_key_f(float x) {
  const uint32_t u = __float_as_uint(x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float from_ord_key_f(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// One workgroup per query: keep the pooled entries >= t0 (the k-th largest workgroup maximum, a
// lower bound of the pooled k-th best), sort them, keep k, certify, emit.
// Round 3: the whole pool (16 entries per thread), the lists' bounds and maxima are loaded in one
// round trip before anything waits (was one dependent load per loop trip), t0 comes from a
// one-wave radix select over the maxima (was a 256-entry LDS bitonic sort), and up to 64 kept
// entries are sorted inside one wave.
constexpr int kSmPer = kMaxRanges * kKW / 256;  // pool entries per thread (one round)
__global__ __launch_bounds__(256) void sparse_merge_kernel(
    const float* __restrict__ cand_key, const int32_t* __restrict__ cand_row,
    const float* __restrict__ cand_bound, int n_wg, int q_first, int k, int64_t ordinal_base,
    float* __restrict__ out_scores, int64_t* __restrict__ out_ids,
    int32_t* __restrict__ out_count, uint32_t* __restrict__ flags, float* __restrict__ kth_out) {
  // flags / kth_out are indexed by the query's position within the pass (ql); outputs by qg
  __shared__ float skey[kSelCap];
  __shared__ int32_t srow[kSelCap];
  __shared__ uint32_t umax[256];
  __shared__ float red[8];
  __shared__ float t0s;
  __shared__ int ctr[2];
  const int ql = blockIdx.x;
  const int qg = q_first + ql;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = armi::wave_id();
  if (flags[ql] & ARMI_FLAG_CERTIFIED) return;  // answered by the MFMA filter (kth = +inf)
  const int pool = n_wg * kKW;
  float kk[kSmPer];
  int32_t rw[kSmPer];
#pragma unroll
  for (int j = 0; j < kSmPer; ++j) {
    const int e = tid + 256 * j;
    const size_t src = ((size_t)(e / kKW) * kQB + ql) * kKW + (e % kKW);
    kk[j] = e < pool ? cand_key[src] : kNegInf;
    rw[j] = e < pool ? cand_row[src] : 0;
  }
  float b = tid < n_wg ? cand_bound[(size_t)tid * kQB + ql] : kNegInf;
  // entry g * kKW is list g's maximum (sorted lists): entry j = 0 of thread tid for g = tid / 16
  // when kKW divides 256; write every list's maximum from the thread that holds it
#pragma unroll
  for (int j = 0; j < kSmPer; ++j) {
    const int e = tid + 256 * j;
    if (e < pool && e % kKW == 0) umax[e / kKW] = ord_key_f(kk[j]);
  }
  if (tid == 0) ctr[0] = 0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) b = fmaxf(b, armi::xor_stride(b, off));
  if (lane == 0) red[wave] = b;
  __syncthreads();
  if (wave == 0) {  // t0 = k-th largest list maximum (radix select over <= 256 keys)
    uint32_t u[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int g = lane + 64 * i;
      u[i] = g < n_wg ? umax[g] : ord_key_f(kNegInf);
    }
    float t0 = kNegInf;
    if (n_wg >= k) {
      uint32_t prefix = 0;
      for (int bit = 31; bit >= 0; --bit) {
        const uint32_t cand = prefix | (1u << bit);
        int cnt = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) cnt += __popcll(__ballot(u[i] >= cand));
        if (cnt >= k) prefix = cand;
      }
      t0 = from_ord_key_f(prefix);
    }
    if (lane == 0) t0s = t0;
  }
  __syncthreads();
  const float t0 = t0s;
  float dmax = kNegInf;
#pragma unroll
  for (int j = 0; j < kSmPer; ++j) {
    if (kk[j] == kNegInf) continue;
    if (kk[j] >= t0) {
      const int slot = atomicAdd(&ctr[0], 1);
      if (slot < kSelCap) {
        skey[slot] = kk[j];
        srow[slot] = rw[j];
      }
    } else {
      dmax = fmaxf(dmax, kk[j]);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) dmax = fmaxf(dmax, armi::xor_stride(dmax, off));
  if (lane == 0) red[4 + wave] = dmax;
  __syncthreads();
  const int n_sel = ctr[0];
  const bool overflow = n_sel > kSelCap;
  const int n_keep = overflow ? kSelCap : n_sel;
  int n2 = armi::pow2_at_least(max(n_keep, max(k, 2)));
  if (n2 <= 64) {
    n2 = 64;
    if (wave == 0) {
      float key = lane < n_keep ? skey[lane] : kNegInf;
      int32_t row = lane < n_keep ? srow[lane] : 0x7fffffff;
      armi::wave_sort_approx_desc(key, row);
      skey[lane] = key;
      srow[lane] = row;
    }
    __syncthreads();
  } else {
    for (int e = n_keep + tid; e < n2; e += 256) {
      skey[e] = kNegInf;
      srow[e] = 0x7fffffff;
    }
    armi::lds_sort_approx_desc(skey, srow, n2);
  }
  float bound = red[0];
#pragma unroll
  for (int w = 1; w < 8; ++w) bound = fmaxf(bound, red[w]);
  if (n2 > k) bound = fmaxf(bound, skey[k]);
  if (wave != 0) return;
  // valid entries form a prefix of the sorted list
  int nv = 0;
  for (int c = lane; c < min(n2, k); c += 64) nv += skey[c] != kNegInf;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) nv += armi::xor_stride(nv, off);
  bool certified;
  if (nv >= k)
    certified = skey[k - 1] > bound;
  else
    certified = (bound == kNegInf);
  certified = certified && !overflow;
  if (certified) {
    for (int c = lane; c < k; c += 64) {
      const size_t o = (size_t)qg * k + c;
      out_scores[o] = c < nv ? skey[c] : kNegInf;
      out_ids[o] = c < nv ? ordinal_base + srow[c] : -1;
    }
  }
  if (lane == 0) {
    out_count[qg] = certified ? nv : 0;
    flags[ql] |= certified ? ARMI_FLAG_CERTIFIED : 0u;
    // collection threshold of the fallback: the k-th candidate (a lower bound of the true k-th);
    // -inf when fewer than k candidates exist
    kth_out[ql] = certified ? std::numeric_limits<float>::infinity()
                            : (nv >= k ? skey[k - 1] : kNegInf);
  }
}

// Second-pass merge, one workgroup per query of the pass (certified queries exit at once): sort
// the rows the collect pass appended (every row scoring >= the k-th candidate) and keep k.
// A list that overflowed (more than kCollectCap rows reach the threshold: a pile of re-uploaded
// identical chunks, or a threshold of -inf when the merge held fewer than k candidates) is
// answered by the grid's n_help helper workgroups instead, exactly: helper h scores its 1/n_help
// of the shard's rows for that query, term at a time in ascending term order (fl32(w * v) added
// to an fp32 sum that starts at 0: the scan's sum, whose absent terms add +-0), keeps its slice's
// top k by (score desc, row asc) and writes them into the query's collect list at slot h * k;
// the last helper to finish (a per-query counter, zeroed with the collect counts) sorts those
// n_help * k <= kCollectCap rows and emits the top k. On calls without an overflowed list the
// helpers check every query's count at once and exit.
constexpr int kHelpRows = 4096;                // rows a helper scores per chunk
constexpr int kHelpPer = kHelpRows / 256;      // ... per thread (thread t owns rows t + 256 i)
constexpr int kMaxHelp = 64;
constexpr int kBestPad = 256;                  // the running best list (>= kMaxK entries)
constexpr int kHelpSort = 8192;                // >= kBestPad + kHelpRows, a power of 2
static_assert(kBestPad >= kMaxK && kHelpSort >= kBestPad + kHelpRows, "helper sort buffer");
static_assert(kHelpSort >= kCollectCap, "the collect list sorts in the same buffer");
// sort buffer (key f32, row i32), chunk accumulators, chunk row flags, per-term weight / dense
// column / cursor / list end, small shared words
constexpr size_t kCollectLds =
    (size_t)kHelpSort * 8 + kHelpRows * 4 + kHelpRows + (size_t)kMaxTerms * 16 + 64;

__global__ __launch_bounds__(256) void sparse_collect_merge_kernel(
    const int* __restrict__ coll_count, float* __restrict__ coll_key,
    int32_t* __restrict__ coll_row, int* __restrict__ help_done, int nq, int q_first, int k,
    int64_t ordinal_base, int64_t n_rows, const uint64_t* __restrict__ row_mask,
    const int32_t* __restrict__ term_ptr, const int2* __restrict__ post,
    const int32_t* __restrict__ dense_of, const uint32_t* __restrict__ dense_val,
    int64_t dense_stride, const int32_t* __restrict__ uterm, const QTerm* __restrict__ qlist,
    const int32_t* __restrict__ qu, const int32_t* __restrict__ qcount,
    const int32_t* __restrict__ qof, float* __restrict__ out_scores,
    int64_t* __restrict__ out_ids, int32_t* __restrict__ out_count, uint32_t* __restrict__ flags) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* skey = reinterpret_cast<float*>(smem);                      // [kHelpSort]
  int32_t* srow = reinterpret_cast<int32_t*>(smem + kHelpSort * 4);  // [kHelpSort]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = armi::wave_id();
  // emit the sorted [0, k) of skey / srow for query ql (valid entries form a prefix)
  auto write_out = [&](int ql) {
    if (wave != 0) return;
    int nv = 0;
    for (int c = lane; c < k; c += 64) nv += srow[c] != kEndRow;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) nv += armi::xor_stride(nv, off);
    const int qg = q_first + ql;
    for (int c = lane; c < k; c += 64) {
      const size_t o = (size_t)qg * k + c;
      out_scores[o] = c < nv ? skey[c] : kNegInf;
      out_ids[o] = c < nv ? ordinal_base + srow[c] : -1;
    }
    if (lane == 0) {
      out_count[qg] = nv;
      flags[ql] |= ARMI_FLAG_FALLBACK;
    }
  };
  if ((int)blockIdx.x < nq) {  // the query's own workgroup
    const int ql = blockIdx.x;
    if (flags[ql] & ARMI_FLAG_CERTIFIED) return;  // workgroup-uniform
    const int total = coll_count[ql];
    if (total > kCollectCap) return;  // overflowed: the helpers answer it
    const int n2 = armi::pow2_at_least(max(max(total, k), 2));
    for (int e = tid; e < n2; e += 256) {
      skey[e] = e < total ? coll_key[(size_t)ql * kCollectCap + e] : kNegInf;
      srow[e] = e < total ? coll_row[(size_t)ql * kCollectCap + e] : kEndRow;
    }
    armi::lds_sort_approx_desc(skey, srow, n2);
    __syncthreads();
    write_out(ql);
    return;
  }
  const int n_help = (int)gridDim.x - nq;
  const int h = (int)blockIdx.x - nq;
  bool any = false;
  for (int q = tid; q < nq; q += 256)
    any |= !(flags[q] & ARMI_FLAG_CERTIFIED) && coll_count[q] > kCollectCap;
  if (!__syncthreads_or(any)) return;  // workgroup-uniform
  float* acc = reinterpret_cast<float*>(smem + kHelpSort * 8);                  // [kHelpRows]
  uint8_t* has = smem + kHelpSort * 8 + kHelpRows * 4;                          // [kHelpRows]
  float* tw = reinterpret_cast<float*>(has + kHelpRows);                        // [kMaxTerms]
  int32_t* tcol = reinterpret_cast<int32_t*>(tw + kMaxTerms);                   // [kMaxTerms]
  int32_t* tcur = tcol + kMaxTerms;                                             // [kMaxTerms]
  int32_t* tend = tcur + kMaxTerms;                                             // [kMaxTerms]
  int* sh = reinterpret_cast<int*>(tend + kMaxTerms);  // [0] slot, [1] survivors, [2] last helper
  const int64_t lo = n_rows * h / n_help, hi = n_rows * (h + 1) / n_help;
  for (int ql = 0; ql < nq; ++ql) {
    if ((flags[ql] & ARMI_FLAG_CERTIFIED) || coll_count[ql] <= kCollectCap) continue;  // uniform
    __syncthreads();  // the previous query is done with the shared arrays
    if (tid < kQB && qof[tid] == ql) sh[0] = tid;
    for (int e = tid; e < kBestPad; e += 256) {
      skey[e] = kNegInf;
      srow[e] = kEndRow;
    }
    __syncthreads();
    const int slot = sh[0];
    const int nt = qcount[slot];
    for (int j = tid; j < nt; j += 256) {  // the query's terms, ascending
      const int32_t t = uterm[qu[slot * kQStride + j]];
      tw[j] = qlist[slot * kQStride + j].w;
      const int32_t d = dense_of[t];
      tcol[j] = d;
      // non-dense term: its first posting at or after row lo, and its list's sentinel
      const int32_t b = term_ptr[t], e = term_ptr[t + 1] - 1;
      int32_t a = b, n = d >= 0 ? 0 : e - b;
      while (n > 0) {
        const int32_t hh = n >> 1;
        if (post[a + hh].x < lo) {
          a += hh + 1;
          n -= hh + 1;
        } else {
          n = hh;
        }
      }
      tcur[j] = a;
      tend[j] = e;
    }
    __syncthreads();
    for (int64_t c0 = lo; c0 < hi; c0 += kHelpRows) {
      const int32_t chi = (int32_t)min<int64_t>(c0 + kHelpRows, hi);
      const int32_t r0 = (int32_t)c0;
#pragma unroll
      for (int i = 0; i < kHelpPer; ++i) {  // owner-local clear
        acc[tid + 256 * i] = 0.f;
        has[tid + 256 * i] = 0;
      }
      bool scattered = false;  // a posting term wrote other threads' rows since the last barrier
      for (int j = 0; j < nt; ++j) {
        const int32_t d = tcol[j];
        const float w = tw[j];
        if (d >= 0) {  // dense column: each thread adds to its own rows, no barrier between terms
          if (scattered) {
            __syncthreads();
            scattered = false;
          }
          const uint32_t* col = dense_val + (size_t)d * dense_stride;
          uint32_t v[kHelpPer];
#pragma unroll
          for (int i = 0; i < kHelpPer; ++i) {
            const int32_t r = r0 + tid + 256 * i;
            v[i] = r < chi ? col[r] : 0u;
          }
#pragma unroll
          for (int i = 0; i < kHelpPer; ++i) {
            if (v[i] != 0u) {  // 0 = no posting (a zero value is stored as -0.0)
              const int e = tid + 256 * i;
              acc[e] = acc[e] + w * __uint_as_float(v[i]);
              has[e] = 1;
            }
          }
        } else {  // postings: the chunk's ones are a prefix from the cursor (rows ascend)
          __syncthreads();
          int32_t cur = tcur[j];
          const int32_t end = tend[j];
          for (;;) {
            const int32_t e = cur + tid;
            const int2 p = e < end ? post[e] : make_int2(kEndRow, 0);
            const bool in = p.x < chi;
            if (in) {
              const int r = p.x - r0;
              acc[r] = acc[r] + w * __int_as_float(p.y);
              has[r] = 1;
            }
            const int n_in = __syncthreads_count(in);
            cur += n_in;
            if (n_in < 256) break;
          }
          if (tid == 0) tcur[j] = cur;  // read again after the next chunk's barriers
          scattered = true;
        }
      }
      if (tid == 0) sh[1] = 0;
      __syncthreads();
      // rows better than the running k-th (key desc, row asc) join the best list
      const float kk = skey[k - 1];
      const int32_t kr = srow[k - 1];
#pragma unroll
      for (int i = 0; i < kHelpPer; ++i) {
        const int e = tid + 256 * i;
        const int32_t r = r0 + e;
        const bool on = r < chi && has[e] &&
                        (!row_mask || ((row_mask[r >> 6] >> (r & 63)) & 1ull));
        if (on && armi::approx_better(acc[e], r, kk, kr)) {
          const int s2 = atomicAdd(&sh[1], 1);
          skey[kBestPad + s2] = acc[e];
          srow[kBestPad + s2] = r;
        }
      }
      __syncthreads();
      const int ns = sh[1];
      if (ns > 0) {  // uniform
        const int n2 = armi::pow2_at_least(kBestPad + ns);
        for (int e = kBestPad + ns + tid; e < n2; e += 256) {
          skey[e] = kNegInf;
          srow[e] = kEndRow;
        }
        armi::lds_sort_approx_desc(skey, srow, n2);
        __syncthreads();
        for (int e = k + tid; e < kBestPad; e += 256) {
          skey[e] = kNegInf;
          srow[e] = kEndRow;
        }
        __syncthreads();
      }
    }
    // this slice's top k into the query's list, then the last helper merges the slices
    for (int c = tid; c < k; c += 256) {
      coll_key[(size_t)ql * kCollectCap + h * k + c] = skey[c];
      coll_row[(size_t)ql * kCollectCap + h * k + c] = srow[c];
    }
    __threadfence();
    __syncthreads();
    if (tid == 0) sh[2] = atomicAdd(help_done + ql, 1) == n_help - 1;
    __syncthreads();
    if (sh[2]) {
      __threadfence();
      const int m = n_help * k;
      const int n2 = armi::pow2_at_least(max(m, 2));
      for (int e = tid; e < n2; e += 256) {
        skey[e] = e < m ? coll_key[(size_t)ql * kCollectCap + e] : kNegInf;
        srow[e] = e < m ? coll_row[(size_t)ql * kCollectCap + e] : kEndRow;
      }
      armi::lds_sort_approx_desc(skey, srow, n2);
      __syncthreads();
      write_out(ql);
    }
  }
}

#include "sparse_filter.h"

struct Workspace {
  int32_t* uterm;
  int32_t* n_terms;
  QTerm* ql;
  int32_t* qu;
  int32_t* qcount;
  int32_t* qof;
  int2* cursors;
  float* cand_key;
  int32_t* cand_row;
  float* cand_bound;
  float* kth;
  int* coll_count;  // [2 * kQB]: collect counts, then the helpers' done counters
  float* coll_key;
  int32_t* coll_row;
  uint16_t* fB;     // MFMA filter: the pass's B slices [kFMaxSeg][kQB][kFK] fp16
  float* fscale;    // its key scale
  int32_t* felig;   // [kQB] queries the filter may answer
  float* fs;        // FilterPrep's per-entry tables
  int4* fterm;
  float* fw;
  int32_t* fnt;
  size_t bytes;
};

Workspace carve(void* base, const armi_sparse_index* idx) {
  armi::Carver cv(base);
  Workspace w{};
  const size_t nr = (size_t)std::max(idx->n_ranges, 1);
  w.uterm = cv.take<int32_t>(kMaxU);
  w.n_terms = cv.take<int32_t>(1);
  w.ql = cv.take<QTerm>((size_t)kQB * kQStride);
  w.qu = cv.take<int32_t>((size_t)kQB * kQStride);
  w.qcount = cv.take<int32_t>(kQB);
  w.qof = cv.take<int32_t>(kQB);
  w.cursors = cv.take<int2>(nr * kMaxU);
  w.cand_key = cv.take<float>(nr * kQB * kKW);
  w.cand_row = cv.take<int32_t>(nr * kQB * kKW);
  w.cand_bound = cv.take<float>(nr * kQB);
  w.kth = cv.take<float>(kQB);
  w.coll_count = cv.take<int>(2 * kQB);
  w.coll_key = cv.take<float>((size_t)kQB * kCollectCap);
  w.coll_row = cv.take<int32_t>((size_t)kQB * kCollectCap);
  w.fB = cv.take<uint16_t>((size_t)kFMaxSeg * kFBSlice);
  w.fscale = cv.take<float>(1);
  w.felig = cv.take<int32_t>(kQB);
  w.fs = cv.take<float>((size_t)kQB * kQStride);
  w.fterm = cv.take<int4>((size_t)kQB * kMaxTerms);
  w.fw = cv.take<float>((size_t)kQB * kMaxTerms);
  w.fnt = cv.take<int32_t>(kQB);
  w.bytes = cv.off + 256;
  return w;
}

// Device temporaries of the index build, released on every exit path.
struct Scratch {
  std::vector<void*> ptrs;
  template <typename T>
  hipError_t alloc(T** p, size_t count) {
    *p = nullptr;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(p), std::max<size_t>(count, 1) * sizeof(T));
    if (e == hipSuccess) ptrs.push_back(*p);
    return e;
  }
  ~Scratch() {
    for (void* p : ptrs) (void)hipFree(p);
  }
};

unsigned grid_for(int64_t n, int block) { return (unsigned)std::max<int64_t>(1, (n + block - 1) / block); }

int build_inverted(armi_sparse_index* idx, const int64_t* indptr, const int32_t* indices,
                   const float* values, hipStream_t stream) {
  const int64_t nnz = idx->nnz;
  const int32_t vocab = idx->vocab;
  Scratch tmp;
  int32_t *row_of, *ent, *sent, *is_long, *scan;
  uint32_t *keys, *skeys;
  ARMI_HIP(tmp.alloc(&row_of, nnz));
  ARMI_HIP(tmp.alloc(&ent, nnz));
  ARMI_HIP(tmp.alloc(&sent, nnz));
  ARMI_HIP(tmp.alloc(&keys, nnz));
  ARMI_HIP(tmp.alloc(&skeys, nnz));
  ARMI_HIP(tmp.alloc(&is_long, (size_t)vocab + 1));
  ARMI_HIP(tmp.alloc(&scan, (size_t)vocab + 1));
  if (nnz > 0) {
    unsigned long long* bad;
    ARMI_HIP(tmp.alloc(&bad, 1));
    ARMI_HIP(hipMemsetAsync(bad, 0, 8, stream));
    count_nonfinite_kernel<<<grid_for(nnz, 256), 256, 0, stream>>>(values, nnz, bad);
    ARMI_LAUNCHED("count_nonfinite_kernel");
    unsigned long long n_bad = 0;
    ARMI_HIP(hipMemcpyAsync(&n_bad, bad, 8, hipMemcpyDeviceToHost, stream));
    ARMI_HIP(hipStreamSynchronize(stream));
    ARMI_REQUIRE(n_bad == 0, "armi_sparse_index_create: values must be finite");
    entry_rows_kernel<<<grid_for(idx->n_rows, 4), 256, 0, stream>>>(indptr, idx->n_rows, row_of);
    ARMI_LAUNCHED("entry_rows_kernel");
    term_keys_kernel<<<grid_for(nnz, 256), 256, 0, stream>>>(indices, nnz, vocab, keys, ent);
    ARMI_LAUNCHED("term_keys_kernel");
    int end_bit = 1;
    while (end_bit < 32 && (uint64_t(1) << end_bit) <= (uint64_t)vocab) ++end_bit;
    size_t sort_bytes = 0;
    ARMI_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, keys, skeys, ent, sent,
                                                (int)nnz, 0, end_bit, stream));
    unsigned char* sort_tmp;
    ARMI_HIP(tmp.alloc(&sort_tmp, sort_bytes));
    ARMI_HIP(hipcub::DeviceRadixSort::SortPairs(sort_tmp, sort_bytes, keys, skeys, ent, sent,
                                                (int)nnz, 0, end_bit, stream));
  }
  ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&idx->term_ptr), ((size_t)vocab + 1) * 4));
  term_ptr_kernel<<<grid_for(nnz + 1, 256), 256, 0, stream>>>(skeys, nnz, vocab, idx->term_ptr);
  ARMI_LAUNCHED("term_ptr_kernel");
  int32_t n_post = 0;
  ARMI_HIP(hipMemcpyAsync(&n_post, idx->term_ptr + vocab, 4, hipMemcpyDeviceToHost, stream));
  ARMI_HIP(hipStreamSynchronize(stream));
  idx->n_postings = n_post;
  const size_t cap = (size_t)n_post + kPad;
  ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&idx->post), cap * 8));
  if (nnz > 0) {
    postings_kernel<<<grid_for(nnz, 256), 256, 0, stream>>>(skeys, sent, row_of, values, nnz, vocab,
                                                            reinterpret_cast<int2*>(idx->post));
    ARMI_LAUNCHED("postings_kernel");
  }
  sentinels_kernel<<<grid_for(std::max<int64_t>((int64_t)vocab + 1, kPad), 256), 256, 0, stream>>>(
      idx->term_ptr, vocab, idx->n_postings, reinterpret_cast<int2*>(idx->post), is_long);
  ARMI_LAUNCHED("sentinels_kernel");
  size_t scan_bytes = 0;
  ARMI_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, is_long, scan, vocab + 1, stream));
  unsigned char* scan_tmp;
  ARMI_HIP(tmp.alloc(&scan_tmp, scan_bytes));
  ARMI_HIP(hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, is_long, scan, vocab + 1, stream));
  int32_t n_long = 0;
  ARMI_HIP(hipMemcpyAsync(&n_long, scan + vocab, 4, hipMemcpyDeviceToHost, stream));
  ARMI_HIP(hipStreamSynchronize(stream));
  idx->n_long = n_long;
  ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&idx->long_of), std::max<size_t>(vocab, 1) * 4));
  long_of_kernel<<<grid_for(vocab, 256), 256, 0, stream>>>(idx->term_ptr, vocab, scan, idx->long_of);
  ARMI_LAUNCHED("long_of_kernel");
  const size_t tab = std::max<size_t>((size_t)n_long * std::max(idx->n_ranges, 1), 1);
  ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&idx->start_tab), tab * 4));
  if (nnz > 0 && n_long > 0 && idx->n_ranges > 0) {
    start_tab_kernel<<<grid_for(nnz, 256), 256, 0, stream>>>(skeys, nnz, vocab, idx->term_ptr,
                                                             idx->long_of,
                                                             reinterpret_cast<const int2*>(idx->post),
                                                             idx->range_rows, idx->n_ranges,
                                                             idx->start_tab);
    ARMI_LAUNCHED("start_tab_kernel");
  }
  // dense columns (at most 4x the bytes of their postings: df >= rows / 8, 4 B per row)
  int32_t *dflag, *dscan;
  ARMI_HIP(tmp.alloc(&dflag, (size_t)vocab + 1));
  ARMI_HIP(tmp.alloc(&dscan, (size_t)vocab + 1));
  dense_flag_kernel<<<grid_for((int64_t)vocab + 1, 256), 256, 0, stream>>>(idx->term_ptr, vocab,
                                                                          idx->n_rows, dflag);
  ARMI_LAUNCHED("dense_flag_kernel");
  size_t dscan_bytes = 0;
  ARMI_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, dscan_bytes, dflag, dscan, vocab + 1, stream));
  unsigned char* dscan_tmp;
  ARMI_HIP(tmp.alloc(&dscan_tmp, dscan_bytes));
  ARMI_HIP(hipcub::DeviceScan::ExclusiveSum(dscan_tmp, dscan_bytes, dflag, dscan, vocab + 1, stream));
  int32_t n_dense = 0;
  ARMI_HIP(hipMemcpyAsync(&n_dense, dscan + vocab, 4, hipMemcpyDeviceToHost, stream));
  ARMI_HIP(hipStreamSynchronize(stream));
  idx->n_dense = n_dense;
  idx->dense_stride = (idx->n_rows + kTile - 1) / kTile * kTile + kTile;  // + the 16-B over-read
  ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&idx->dense_of), std::max<size_t>(vocab, 1) * 4));
  dense_of_kernel<<<grid_for(vocab, 256), 256, 0, stream>>>(dflag, dscan, vocab, idx->dense_of);
  ARMI_LAUNCHED("dense_of_kernel");
  const size_t dense_words = std::max<size_t>((size_t)n_dense * idx->dense_stride, 1);
  ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&idx->dense_val), dense_words * 4));
  ARMI_HIP(hipMemsetAsync(idx->dense_val, 0, dense_words * 4, stream));
  if (nnz > 0 && n_dense > 0) {
    dense_fill_kernel<<<grid_for(nnz, 256), 256, 0, stream>>>(
        idx->term_ptr, idx->dense_of, reinterpret_cast<const int2*>(idx->post), idx->n_postings,
        skeys, nnz, vocab, idx->dense_stride, idx->dense_val);
    ARMI_LAUNCHED("dense_fill_kernel");
  }
  // the filter rescore's rare-value tables (sparse_filter.h): every posting of a term without an
  // fp32 column; on an insert that finds both buckets full, again with twice the buckets
  {
    int32_t *nb, *nbscan, *fail;
    ARMI_HIP(tmp.alloc(&nb, (size_t)vocab + 1));
    ARMI_HIP(tmp.alloc(&nbscan, (size_t)vocab + 1));
    ARMI_HIP(tmp.alloc(&fail, 1));
    ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&idx->rare_of), std::max<size_t>(vocab, 1) * 8));
    // (ARMI_RARE_DIV, a test knob: postings per bucket targeted, default 4; tests raise it to
    // force full bucket pairs and the overflow chains)
    const char* dv = getenv("ARMI_RARE_DIV");
    for (int div = dv ? std::max(1, atoi(dv)) : 4;; div /= 2) {
      rare_buckets_kernel<<<grid_for((int64_t)vocab + 1, 256), 256, 0, stream>>>(
          idx->term_ptr, idx->dense_of, vocab, div, nb);
      ARMI_LAUNCHED("rare_buckets_kernel");
      ARMI_HIP(hipcub::DeviceScan::ExclusiveSum(dscan_tmp, dscan_bytes, nb, nbscan, vocab + 1, stream));
      int32_t n_buckets = 0;
      ARMI_HIP(hipMemcpyAsync(&n_buckets, nbscan + vocab, 4, hipMemcpyDeviceToHost, stream));
      ARMI_HIP(hipStreamSynchronize(stream));
      rare_of_kernel<<<grid_for(vocab, 256), 256, 0, stream>>>(nb, nbscan, vocab, idx->rare_of);
      ARMI_LAUNCHED("rare_of_kernel");
      if (idx->rare_tab) ARMI_HIP(hipFree(idx->rare_tab));
      idx->rare_tab = nullptr;
      const size_t slots = std::max<size_t>((size_t)n_buckets * kRareSlots, 1);
      ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&idx->rare_tab), slots * 8));
      ARMI_HIP(hipMemsetAsync(idx->rare_tab, 0xff, slots * 8, stream));
      ARMI_HIP(hipMemsetAsync(fail, 0, 4, stream));
      if (nnz > 0 && n_buckets > 0) {
        int32_t* fill;
        ARMI_HIP(tmp.alloc(&fill, (size_t)n_buckets));
        ARMI_HIP(hipMemsetAsync(fill, 0, (size_t)n_buckets * 4, stream));
        rare_insert_kernel<<<grid_for(nnz, 256), 256, 0, stream>>>(
            idx->rare_of, reinterpret_cast<const int2*>(idx->post), skeys, nnz, vocab, fill,
            idx->rare_tab, fail);
        ARMI_LAUNCHED("rare_insert_kernel");
      }
      int32_t failed = 0;
      ARMI_HIP(hipMemcpyAsync(&failed, fail, 4, hipMemcpyDeviceToHost, stream));
      ARMI_HIP(hipStreamSynchronize(stream));
      idx->rare_slots = (int64_t)slots;
      if (failed == 0) break;
      ARMI_REQUIRE(div > 1, "armi_sparse_index: rare-value tables overflow");
    }
  }
  // MFMA filter (sparse_filter.h): per-term scales, u8 columns of the terms in >= 1/32 of the rows
  uint32_t* tmax;
  unsigned long long* n_neg;
  ARMI_HIP(tmp.alloc(&tmax, (size_t)vocab + 1));
  ARMI_HIP(tmp.alloc(&n_neg, 1));
  ARMI_HIP(hipMemsetAsync(tmax, 0, ((size_t)vocab + 1) * 4, stream));
  ARMI_HIP(hipMemsetAsync(n_neg, 0, 8, stream));
  if (nnz > 0) {
    term_max_kernel<<<grid_for(nnz, 256), 256, 0, stream>>>(
        skeys, reinterpret_cast<const int2*>(idx->post), nnz, vocab, tmax, n_neg);
    ARMI_LAUNCHED("term_max_kernel");
  }
  ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&idx->term_scale), std::max<size_t>(vocab, 1) * 4));
  term_scale_kernel<<<grid_for(vocab, 256), 256, 0, stream>>>(tmax, vocab, idx->term_scale);
  ARMI_LAUNCHED("term_scale_kernel");
  col8_flag_kernel<<<grid_for((int64_t)vocab + 1, 256), 256, 0, stream>>>(idx->term_ptr, vocab,
                                                                         idx->n_rows, dflag);
  ARMI_LAUNCHED("col8_flag_kernel");
  ARMI_HIP(hipcub::DeviceScan::ExclusiveSum(dscan_tmp, dscan_bytes, dflag, dscan, vocab + 1, stream));
  int32_t n_col8 = 0;
  ARMI_HIP(hipMemcpyAsync(&n_col8, dscan + vocab, 4, hipMemcpyDeviceToHost, stream));
  ARMI_HIP(hipStreamSynchronize(stream));
  idx->n_col8 = n_col8;
  ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&idx->col8_of), std::max<size_t>(vocab, 1) * 4));
  dense_of_kernel<<<grid_for(vocab, 256), 256, 0, stream>>>(dflag, dscan, vocab, idx->col8_of);
  ARMI_LAUNCHED("dense_of_kernel");
  idx->dense8_stride = (idx->n_rows + kFT - 1) / kFT * kFT + kFT;  // + the last tile's over-read
  const size_t u8_bytes = std::max<size_t>((size_t)n_col8 * idx->dense8_stride, 16);
  ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&idx->dense_u8), u8_bytes));
  ARMI_HIP(hipMemsetAsync(idx->dense_u8, 0, u8_bytes, stream));
  if (nnz > 0 && n_col8 > 0) {
    dense_u8_fill_kernel<<<grid_for(nnz, 256), 256, 0, stream>>>(
        idx->col8_of, reinterpret_cast<const int2*>(idx->post), skeys, nnz, vocab,
        idx->term_scale, idx->dense8_stride, idx->dense_u8);
    ARMI_LAUNCHED("dense_u8_fill_kernel");
  }
  unsigned long long negatives = 0;
  ARMI_HIP(hipMemcpyAsync(&negatives, n_neg, 8, hipMemcpyDeviceToHost, stream));
  ARMI_HIP(hipStreamSynchronize(stream));
  idx->filter_ok = negatives == 0;
  idx->filter_on = true;
  return ARMI_OK;
}

void free_index(armi_sparse_index* idx) {
  (void)hipFree(idx->term_ptr);
  (void)hipFree(idx->post);
  (void)hipFree(idx->long_of);
  (void)hipFree(idx->start_tab);
  (void)hipFree(idx->dense_of);
  (void)hipFree(idx->dense_val);
  (void)hipFree(idx->term_scale);
  (void)hipFree(idx->dense_u8);
  (void)hipFree(idx->col8_of);
  (void)hipFree(idx->rare_of);
  (void)hipFree(idx->rare_tab);
  delete idx;
}

// Sparse query CSR <-> fixed slots, the query exchange of a sharded hybrid step (each query's
// terms padded to `slots` entries, so every rank knows the all-gather's size without a host sync).
// Pack: one thread per (query, slot); terms past `slots` are dropped (callers refuse such queries
// first). Unpack: one workgroup reads the gathered rows in place (byte row stride, field offsets),
// prefix-sums the counts and copies each query's live slots into a CSR.
__global__ __launch_bounds__(256) void query_slots_pack_kernel(
    const int32_t* __restrict__ indptr, const int32_t* __restrict__ idx,
    const float* __restrict__ val, int n, int slots, int32_t* __restrict__ count,
    int32_t* __restrict__ sidx, float* __restrict__ sval) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)n * slots) return;
  const int q = (int)(e / slots), j = (int)(e % slots);
  const int32_t a = indptr[q];
  const int32_t c = min(indptr[q + 1] - a, slots);
  if (j == 0) count[q] = c;
  sidx[e] = j < c ? idx[a + j] : 0;
  sval[e] = j < c ? val[a + j] : 0.0f;
}

constexpr int kUnpackThreads = 1024;
__global__ __launch_bounds__(kUnpackThreads) void query_slots_unpack_kernel(
    const unsigned char* __restrict__ rows, int64_t row_stride, int64_t off_count,
    int64_t off_idx, int64_t off_val, int n, int slots, int32_t* __restrict__ indptr,
    int32_t* __restrict__ idx, float* __restrict__ val) {
  __shared__ int32_t wsum[kUnpackThreads / 64];
  __shared__ int32_t carry;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) {
    carry = 0;
    indptr[0] = 0;
  }
  __syncthreads();
  for (int q0 = 0; q0 < n; q0 += kUnpackThreads) {
    const int q = q0 + tid;
    const int32_t c =
        q < n ? min(max(*reinterpret_cast<const int32_t*>(rows + q * row_stride + off_count), 0),
                    slots)
              : 0;
    int32_t x = c;  // inclusive wave scan
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int32_t y = __shfl_up(x, off);
      if (lane >= off) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    int32_t before = carry;
    for (int w = 0; w < wave; ++w) before += wsum[w];
    const int32_t start = before + x - c;
    if (q < n) {
      indptr[q + 1] = start + c;
      const int32_t* si = reinterpret_cast<const int32_t*>(rows + q * row_stride + off_idx);
      const float* sv = reinterpret_cast<const float*>(rows + q * row_stride + off_val);
      for (int j = 0; j < c; ++j) {
        idx[start + j] = si[j];
        val[start + j] = sv[j];
      }
    }
    __syncthreads();
    if (tid == kUnpackThreads - 1) carry = start + c;
    __syncthreads();
  }
}

}  // namespace

extern "C" {

int armi_sparse_index_create(int device, const int64_t* indptr, const int32_t* indices,
                             const float* values, int64_t n_rows, int64_t nnz, int32_t vocab,
                             int64_t ordinal_base, armi_sparse_index** out, hipStream_t stream) {
  ARMI_REQUIRE(out != nullptr, "armi_sparse_index_create: out is null");
  *out = nullptr;
  ARMI_REQUIRE(n_rows >= 0 && n_rows < (int64_t(1) << 31) - 64,
               "armi_sparse_index_create: bad n_rows");
  ARMI_REQUIRE(vocab >= 1 && vocab < (1 << 26), "armi_sparse_index_create: vocab must be in [1, 2^26)");
  ARMI_REQUIRE(nnz >= 0 && nnz + (int64_t)vocab + kPad < (int64_t(1) << 31),
               "armi_sparse_index_create: nnz + vocab must stay below 2^31");
  ARMI_REQUIRE(indptr != nullptr || n_rows == 0, "armi_sparse_index_create: indptr is null");
  ARMI_REQUIRE((indices && values) || nnz == 0, "armi_sparse_index_create: null CSR arrays");
  ARMI_HIP(hipSetDevice(device));
  hipDeviceProp_t prop;
  ARMI_HIP(hipGetDeviceProperties(&prop, device));
  armi_sparse_index* idx = new armi_sparse_index();
  idx->device = device;
  idx->n_rows = n_rows;
  idx->nnz = nnz;
  idx->vocab = vocab;
  idx->ordinal_base = ordinal_base;
  idx->num_cus = prop.multiProcessorCount;
  if (n_rows > 0) {
    const int64_t want = std::max<int64_t>(
        1, std::min<int64_t>(std::min(idx->num_cus, kMaxRanges), (n_rows + 63) / 64));
    idx->range_rows = ((n_rows + want - 1) / want + 63) / 64 * 64;
    idx->n_ranges = (int)((n_rows + idx->range_rows - 1) / idx->range_rows);
  } else {
    idx->range_rows = 64;
    idx->n_ranges = 0;
  }
  const int rc = build_inverted(idx, indptr, indices, values, stream);
  if (rc != ARMI_OK) {
    free_index(idx);
    return rc;
  }
  *out = idx;
  return ARMI_OK;
}

int armi_sparse_index_destroy(armi_sparse_index* index) {
  if (index) {
    (void)hipSetDevice(index->device);
    free_index(index);
  }
  return ARMI_OK;
}

size_t armi_sparse_workspace_bytes(const armi_sparse_index* idx, int n_queries, int k) {
  (void)k;
  if (!idx || n_queries <= 0) return 0;
  return carve(nullptr, idx).bytes;
}

int armi_sparse_topk(const armi_sparse_index* idx, const int32_t* q_indptr,
                     const int32_t* q_indices, const float* q_values, int n_queries, int k,
                     const uint64_t* row_mask, float* out_scores, int64_t* out_ids,
                     int32_t* out_count, uint32_t* out_flags, void* workspace,
                     size_t workspace_bytes, hipStream_t stream) {
  ARMI_REQUIRE(idx != nullptr, "armi_sparse_topk: index is null");
  ARMI_REQUIRE(k >= 1 && k <= kMaxK, "armi_sparse_topk: k must be in [1, 240]");
  if (n_queries <= 0) return ARMI_OK;
  ARMI_REQUIRE(q_indptr && q_indices && q_values && out_scores && out_ids && out_count &&
                   out_flags && workspace,
               "armi_sparse_topk: null pointer argument");
  ARMI_REQUIRE(workspace_bytes >= armi_sparse_workspace_bytes(idx, n_queries, k),
               "armi_sparse_topk: workspace too small");
  ARMI_HIP(hipSetDevice(idx->device));
  const Workspace w = carve(workspace, idx);
#ifdef ARMI_SPARSE_PROFILE
  static const int dbg = getenv("ARMI_SPARSE_DBG") ? atoi(getenv("ARMI_SPARSE_DBG")) : 0;
#else
  constexpr int dbg = 0;
#endif
  // dynamic-LDS limits raised once per device (no runtime calls but stream work per search:
  // graph-capturable)
  if (int rc = armi::allow_lds(sparse_collect_merge_kernel, kCollectLds)) return rc;
  if (int rc = armi::allow_lds(pass_terms_kernel, kPrepLds)) return rc;
  if (int rc = armi::allow_lds(pass_terms_bitmap_kernel, kPrepBmLds)) return rc;
  if (int rc = armi::allow_lds(sparse_scan_kernel<false>, kScanLds)) return rc;
  if (int rc = armi::allow_lds(sparse_scan_kernel<true>, kScanLds)) return rc;
  if (int rc = armi::allow_lds(sparse_filter_scan_kernel, kFLds)) return rc;
  const int n_help = std::max(1, std::min(kMaxHelp, kCollectCap / k));
  // the MFMA filter answers what it can certify; kc = the rescored candidates per query
  const bool filter = idx->filter_ok && idx->filter_on && k <= kFMaxK && idx->n_ranges > 0;
  const int kc = std::min(kFSel / 2, std::max(k + 32, 2 * k));
  armi::TimedLaunch stage;
  // (a call whose whole stage is timed does not also time its scan: the scan's event-bound
  // dispatch would inflate the stage; with a timing period of 2 the two alternate)
  const int stage_timed = stage.begin(ARMI_TIMING_SPARSE_STAGE, stream);
  if (stage_timed < 0) return ARMI_ERR_HIP;
  const int scan_slot = stage_timed ? -1 : ARMI_TIMING_SPARSE_SCAN;
  for (int q0 = 0; q0 < n_queries; q0 += kQB) {
    const int nqp = std::min(kQB, n_queries - q0);
    uint32_t* pflags = out_flags + q0;
    if (idx->n_rows == 0) {
      ARMI_HIP(hipMemsetAsync(out_count + q0, 0, sizeof(int32_t) * nqp, stream));
      ARMI_HIP(hipMemsetAsync(pflags, 0, sizeof(uint32_t) * nqp, stream));
      ARMI_HIP(hipMemsetAsync(out_ids + (size_t)q0 * k, 0xff, sizeof(int64_t) * nqp * k, stream));
      continue;
    }
    // (with the filter on, the pass_terms block also writes the filter's B slices)
    const FilterPrep fp{idx->term_scale, idx->dense_of, idx->rare_of,
                        filter ? w.fB : nullptr, w.fscale, w.felig, w.fs, w.fterm, w.fw, w.fnt};
    if (idx->vocab <= kBitmapVocab)
      pass_terms_bitmap_kernel<<<dim3(1), dim3(kScanThreads), kPrepBmLds, stream>>>(
          q_indptr + q0, q_indices, q_values, nqp, idx->vocab, w.uterm, w.n_terms, w.ql, w.qu,
          w.qcount, w.qof, pflags, w.coll_count, fp);
    else
      pass_terms_kernel<<<dim3(1), dim3(1024), kPrepLds, stream>>>(
          q_indptr + q0, q_indices, q_values, nqp, idx->vocab, w.uterm, w.n_terms, w.ql, w.qu,
          w.qcount, w.qof, pflags, w.coll_count, fp);
    ARMI_LAUNCHED("pass_terms_kernel");
    if (filter) {
      const int rc_f = armi::timed_kernel(
          scan_slot, sparse_filter_scan_kernel, dim3(idx->n_ranges), dim3(kFThreads),
          kFLds, stream, (const int32_t*)idx->term_ptr, reinterpret_cast<const int2*>(idx->post),
          (const int32_t*)idx->long_of, (const int32_t*)idx->start_tab, idx->n_rows,
          idx->range_rows, idx->n_ranges, row_mask, (const int32_t*)w.uterm,
          (const int32_t*)w.n_terms, (const int32_t*)idx->col8_of, (const uint8_t*)idx->dense_u8,
          idx->dense8_stride, (const float*)idx->term_scale, (const uint16_t*)w.fB,
          (const float*)w.fscale, w.cand_key, w.cand_row, w.cand_bound);
      ARMI_LAUNCHED("sparse_filter_scan_kernel");
      if (rc_f) return rc_f;
      sparse_filter_merge_kernel<<<dim3(nqp), dim3(256), 0, stream>>>(
          w.cand_key, w.cand_row, w.cand_bound, idx->n_ranges, q0, k, kc, idx->ordinal_base,
          w.felig, w.fterm, w.fw, w.fnt, idx->rare_tab, idx->dense_val, idx->dense_stride,
          out_scores, out_ids, out_count, pflags, w.kth);
      ARMI_LAUNCHED("sparse_filter_merge_kernel");
#ifdef ARMI_SPARSE_PROFILE
      if (dbg & 8) {
        std::vector<unsigned long long> hs((size_t)kMaxRanges * kFWaves * 8), hm((size_t)kQB * 16);
        ARMI_HIP(hipStreamSynchronize(stream));
        ARMI_HIP(hipMemcpyFromSymbol(hs.data(), HIP_SYMBOL(g_fscan_prof), hs.size() * 8));
        ARMI_HIP(hipMemcpyFromSymbol(hm.data(), HIP_SYMBOL(g_fmerge_prof), hm.size() * 8));
        double sum[6] = {0}, mx[6] = {0};
        int cnt = 0;
        for (size_t wv = 0; wv < (size_t)idx->n_ranges * kFWaves; ++wv) {
          ++cnt;
          for (int i = 0; i < 6; ++i) {
            sum[i] += (double)hs[wv * 8 + i];
            mx[i] = std::max(mx[i], (double)hs[wv * 8 + i]);
          }
        }
        fprintf(stderr, "filter scan (us) avg/max per wave: issue %.1f/%.1f compute %.1f/%.1f epilogue "
                "%.1f/%.1f finish %.1f/%.1f barrier %.1f/%.1f prologue %.1f/%.1f steps %llu\n",
                sum[0] / cnt / 100, mx[0] / 100, sum[1] / cnt / 100, mx[1] / 100, sum[2] / cnt / 100,
                mx[2] / 100, sum[3] / cnt / 100, mx[3] / 100, sum[4] / cnt / 100, mx[4] / 100,
                sum[5] / cnt / 100, mx[5] / 100, hs[6]);
        double ms[8] = {0};
        int r1 = 0, r2 = 0, fail = 0;
        for (int q = 0; q < nqp; ++q) {
          for (int i = 1; i < 8; ++i) ms[i] += (double)hm[q * 16 + i];
          const long long rr = (long long)hm[q * 16];
          r1 += rr == 1;
          r2 += rr == 2;
          fail += rr < 0;
        }
        double mx7 = 0;
        for (int q = 0; q < nqp; ++q) mx7 = std::max(mx7, (double)hm[q * 16 + 7]);
        std::vector<int> order(nqp);
        for (int q = 0; q < nqp; ++q) order[q] = q;
        std::sort(order.begin(), order.end(),
                  [&](int a, int b) { return hm[a * 16 + 7] > hm[b * 16 + 7]; });
        for (int i = 0; i < std::min(nqp, 6); ++i) {
          const unsigned long long* h = &hm[(size_t)order[i] * 16];
          fprintf(stderr, "  slow query %d: setup %.1f select %.1f rare-start %.1f rescore %.1f rank "
                  "%.1f end %.1f terms %llu rare %llu n_all %llu n_sel %llu\n", order[i],
                  h[1] / 100.0, h[2] / 100.0, h[6] / 100.0, h[3] / 100.0, h[4] / 100.0,
                  h[7] / 100.0, h[8], h[9], h[10], h[11]);
          fprintf(stderr, "    radix %.1f selected %.1f ranked %.1f\n", h[12] / 100.0, h[13] / 100.0,
                  h[14] / 100.0);
        }
        fprintf(stderr, "filter merge (us, stamps from start) avg: setup %.1f select %.1f rescore "
                "%.1f round1 %.1f round2 %.1f end %.1f (max %.1f); rounds 1/2/failed %d/%d/%d\n",
                ms[1] / nqp / 100, ms[2] / nqp / 100, ms[3] / nqp / 100, ms[4] / nqp / 100,
                ms[5] / nqp / 100, ms[7] / nqp / 100, mx7 / 100, r1, r2, fail);
      }
#endif
    }
    // the exact scan: every query when the filter is off, else only the queries it left
    // (the kernel exits at once when it answered all of them)
    armi::TimedLaunch tl;
    if (!filter && tl.begin(scan_slot, stream) < 0) return ARMI_ERR_HIP;
    sparse_scan_kernel<false><<<dim3(idx->n_ranges), dim3(kScanThreads), kScanLds, stream>>>(
        idx->term_ptr, reinterpret_cast<const int2*>(idx->post), idx->long_of, idx->start_tab, idx->n_rows,
        idx->range_rows, idx->n_ranges, row_mask, nqp, w.uterm, w.n_terms, w.ql, w.qu, w.qcount, w.qof,
        w.cursors, w.cand_key, w.cand_row, w.cand_bound, nullptr, nullptr, nullptr, nullptr, dbg,
        idx->dense_of, idx->dense_val, idx->dense_stride, filter ? pflags : nullptr);
    ARMI_LAUNCHED("sparse_scan_kernel");
    if (int rc = tl.end()) return rc;
#ifdef ARMI_SPARSE_PROFILE
    if (dbg & 8) {
      std::vector<unsigned long long> h((size_t)kMaxRanges * kWaves * 12);
      ARMI_HIP(hipStreamSynchronize(stream));
      ARMI_HIP(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_sparse_prof), h.size() * 8));
      double sum[10] = {0}, mx[10] = {0};
      unsigned long long e_min = ~0ull, e_max = 0, x_min = ~0ull, x_max = 0;
      int cnt = 0;
      for (int g = 0; g < idx->n_ranges; ++g)
        for (int wv = 0; wv < kWaves; ++wv) {
          const unsigned long long* pr = &h[((size_t)g * kWaves + wv) * 12];
          ++cnt;
          for (int i = 0; i < 10; ++i) {
            sum[i] += (double)pr[i];
            mx[i] = std::max(mx[i], (double)pr[i]);
          }
          e_min = std::min(e_min, pr[10]);
          e_max = std::max(e_max, pr[10]);
          x_min = std::min(x_min, pr[11]);
          x_max = std::max(x_max, pr[11]);
        }
      fprintf(stderr, "sparse prof (us, 100MHz clock) avg/max: issue %.1f/%.1f compute %.1f/%.1f "
              "cand %.1f/%.1f finish %.1f/%.1f barrier %.1f/%.1f prologue %.1f/%.1f n_w %.1f/%.0f S %.0f "
              "setup %.1f/%.1f tail %.1f/%.1f entry-spread %.1f exit-spread %.1f span %.1f\n",
              sum[0] / cnt / 100, mx[0] / 100, sum[1] / cnt / 100, mx[1] / 100, sum[2] / cnt / 100,
              mx[2] / 100, sum[3] / cnt / 100, mx[3] / 100, sum[4] / cnt / 100, mx[4] / 100,
              sum[5] / cnt / 100, mx[5] / 100, sum[6] / cnt, mx[6], mx[7], sum[8] / cnt / 100,
              mx[8] / 100, sum[9] / cnt / 100, mx[9] / 100, (e_max - e_min) / 100.0,
              (x_max - x_min) / 100.0, (x_max - e_min) / 100.0);
    }
#endif
    sparse_merge_kernel<<<dim3(nqp), dim3(256), 0, stream>>>(
        w.cand_key, w.cand_row, w.cand_bound, idx->n_ranges, q0, k, idx->ordinal_base,
        out_scores, out_ids, out_count, pflags, w.kth);
    ARMI_LAUNCHED("sparse_merge_kernel");
    sparse_scan_kernel<true><<<dim3(idx->n_ranges), dim3(kScanThreads), kScanLds, stream>>>(
        idx->term_ptr, reinterpret_cast<const int2*>(idx->post), idx->long_of, idx->start_tab, idx->n_rows,
        idx->range_rows, idx->n_ranges, row_mask, nqp, w.uterm, w.n_terms, w.ql, w.qu, w.qcount, w.qof,
        w.cursors, nullptr, nullptr, nullptr, w.kth, w.coll_count, w.coll_key, w.coll_row, dbg,
        idx->dense_of, idx->dense_val, idx->dense_stride, nullptr);
    ARMI_LAUNCHED("sparse_collect_kernel");
    sparse_collect_merge_kernel<<<dim3(nqp + n_help), dim3(256), kCollectLds, stream>>>(
        w.coll_count, w.coll_key, w.coll_row, w.coll_count + kQB, nqp, q0,
        k, idx->ordinal_base, idx->n_rows, row_mask, idx->term_ptr,
        reinterpret_cast<const int2*>(idx->post), idx->dense_of, idx->dense_val,
        idx->dense_stride, w.uterm, w.ql, w.qu, w.qcount, w.qof, out_scores, out_ids, out_count,
        pflags);
    ARMI_LAUNCHED("sparse_collect_merge_kernel");
  }
  if (int rc = stage.end()) return rc;
  return ARMI_OK;
}

int armi_sparse_index_set_filter(armi_sparse_index* index, int enable, int* usable) {
  ARMI_REQUIRE(index != nullptr, "armi_sparse_index_set_filter: index is null");
  index->filter_on = enable != 0;
  if (usable) *usable = index->filter_ok ? 1 : 0;
  return ARMI_OK;
}

int armi_query_slots_pack(const int32_t* indptr, const int32_t* indices, const float* values,
                          int n_queries, int slots, int32_t* count, int32_t* slot_indices,
                          float* slot_values, hipStream_t stream) {
  ARMI_REQUIRE(slots >= 1, "armi_query_slots_pack: slots must be >= 1");
  if (n_queries <= 0) return ARMI_OK;
  ARMI_REQUIRE(indptr && indices && values && count && slot_indices && slot_values,
               "armi_query_slots_pack: null pointer argument");
  const int64_t total = (int64_t)n_queries * slots;
  query_slots_pack_kernel<<<dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream>>>(
      indptr, indices, values, n_queries, slots, count, slot_indices, slot_values);
  ARMI_LAUNCHED("query_slots_pack_kernel");
  return ARMI_OK;
}

int armi_query_slots_unpack(const void* rows, int64_t row_stride, int64_t off_count,
                            int64_t off_indices, int64_t off_values, int n_queries, int slots,
                            int32_t* indptr, int32_t* indices, float* values,
                            hipStream_t stream) {
  ARMI_REQUIRE(slots >= 1, "armi_query_slots_unpack: slots must be >= 1");
  ARMI_REQUIRE(rows && indptr && indices && values,
               "armi_query_slots_unpack: null pointer argument");
  const uintptr_t b = reinterpret_cast<uintptr_t>(rows);
  ARMI_REQUIRE(row_stride % 4 == 0 && (b + off_count) % 4 == 0 && (b + off_indices) % 4 == 0 &&
                   (b + off_values) % 4 == 0,
               "armi_query_slots_unpack: fields and row stride must be 4-byte aligned");
  query_slots_unpack_kernel<<<dim3(1), dim3(kUnpackThreads), 0, stream>>>(
      static_cast<const unsigned char*>(rows), row_stride, off_count, off_indices, off_values,
      n_queries < 0 ? 0 : n_queries, slots, indptr, indices, values);
  ARMI_LAUNCHED("query_slots_unpack_kernel");
  return ARMI_OK;
}

}  // extern "C"
