// Sparse lexical-weight top-k over a CSR chunk store (gfx950).
//
// Restates Qdrant's sparse-vector search as called by QdrantRetriever.search
// (src/audio_rag/retrieval/qdrant.py:289-293 sparse prefetch of hybrid search, 299-312 sparse
// query) on the collection's "sparse" vector (SparseVectorParams without IDF modifier,
// qdrant.py:103-107), filled with BGE-M3 lexical weights (embeddings/bge.py:95-102, 122-128):
//   score(q, d) = sum over indices present in both, in ascending index order, of fl32(q_i * d_i)
//   accumulated in fp32 (multiply and add rounded separately; no FMA), only rows that share at
//   least one index are results, ranking (score desc, ordinal asc).
//
// Design (one batch of up to 64 queries per scan; lane l of every wave = query l):
//   prep:   a per-batch term table: slot_of_term[t] = the first (query, term) pair naming t,
//           weights[slot][64] = each query's weight for that term, qmask[slot] = which queries.
//   scan:   row-major walk of the CSR (each byte read once); for every row the wave loads 64
//           (index, value) pairs at a time, looks each index up in slot_of_term, ballots the
//           hits and adds the hits in ascending index order, lane-parallel over queries. Each
//           lane keeps a 4-deep top list of rows for its query plus the best score it dropped.
//   merge:  per query, pool the workgroup lists, keep the k best, certify against the dropped
//           bound (scores are exact, so the bound test is strict: k-th > bound).
//   fallback for uncertified queries: a second scan collects every row scoring >= the k-th
//           candidate (a lower bound of the true k-th), then sorts them.
#include <limits>
#include <vector>

#include "armi_index.h"

namespace {

constexpr int kQB = 64;
constexpr int kLaneList = 4;
constexpr int kScanThreads = 1024;  // 16 waves: one workgroup per CU
constexpr int kWavesPerWG = kScanThreads / 64;
constexpr int kKW = 16;             // candidates per workgroup and query (of 64 lane entries)
constexpr int kSelCap = 1024;       // kept entries per query in the merge
constexpr int kMaxK = 240;
constexpr int kCollectCap = 4096;             // rows per query collected by the fallback
constexpr int kNoSlot = 0x7f7f7f7f;  // byte pattern of the per-pass memset
constexpr float kNegInf = -std::numeric_limits<float>::infinity();
constexpr int64_t kNoOrd = std::numeric_limits<int64_t>::max();
constexpr uint32_t kFlagOverflow = 4u;

constexpr int kMaxTerms = 256;  // query terms per query (BGE-M3 queries are short)

// block per query of the pass: slot_of_term[t] = min pair index (relative to the pass) naming t
__global__ void term_slots_kernel(const int32_t* __restrict__ q_indptr,
                                  const int32_t* __restrict__ q_indices, int32_t vocab,
                                  int32_t* __restrict__ slot_of_term) {
  const int q = blockIdx.x;
  const int32_t base = q_indptr[0];
  const int32_t a = q_indptr[q], e = min(q_indptr[q + 1], a + kMaxTerms);
  for (int32_t p = a + threadIdx.x; p < e; p += blockDim.x) {
    const int32_t t = q_indices[p];
    if (t >= 0 && t < vocab) atomicMin(&slot_of_term[t], p - base);
  }
}

__global__ void term_weights_kernel(const int32_t* __restrict__ q_indptr,
                                    const int32_t* __restrict__ q_indices,
                                    const float* __restrict__ q_values, int32_t vocab,
                                    const int32_t* __restrict__ slot_of_term,
                                    float* __restrict__ weights,
                                    unsigned long long* __restrict__ qmask,
                                    uint32_t* __restrict__ flags) {
  const int q = blockIdx.x;
  const int32_t a = q_indptr[q], b = q_indptr[q + 1];
  const int32_t e = min(b, a + kMaxTerms);
  if (threadIdx.x == 0) flags[q] = (b - a > kMaxTerms) ? 8u : 0u;  // 8 = terms dropped
  for (int32_t p = a + threadIdx.x; p < e; p += blockDim.x) {
    const int32_t t = q_indices[p];
    if (t < 0 || t >= vocab) continue;
    const int s = slot_of_term[t];
    weights[(size_t)s * kQB + q] = q_values[p];
    atomicOr(&qmask[s], 1ull << q);
  }
}

__device__ __forceinline__ void topm_insert(float x, int32_t id, float (&s)[kLaneList],
                                            int32_t (&ix)[kLaneList], float& disc) {
#pragma unroll
  for (int j = 0; j < kLaneList; ++j) {
    // (score desc, row asc): rows arrive in ascending order per lane, so strict > keeps ties
    // in row order
    const bool c = x > s[j];
    const float ts = c ? x : s[j];
    const int32_t ti = c ? id : ix[j];
    x = c ? s[j] : x;
    id = c ? ix[j] : id;
    s[j] = ts;
    ix[j] = ti;
  }
  disc = fmaxf(disc, x);
}

constexpr int kSlots = kQB * kMaxTerms;
constexpr int kHitBatch = 16;

__device__ __forceinline__ int rl_i(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ int64_t rl_64(int64_t v, int lane) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v & 0xffffffffu), lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), lane);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ float rl_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

constexpr uint32_t kAbsent = 0xffffffffu;  // weights[slot][q] bit pattern: q lacks the term

// Walks rows [r0, r1) of the CSR as one flat entry stream [indptr[r0], indptr[r1]), lane l of
// the wave accumulating query l. Per 64-entry block the hit entries (index present in the
// batch's term table) are compacted into this wave's LDS scratch with one mbcnt-ranked write,
// then walked with broadcast LDS reads: no per-hit ballot / readlane scalar work. Loads are
// issued in the order they are consumed (vmcnt retires in issue order): block i's weight loads
// first, then block i+1's term-slot lookups, then block i+2's index / value loads. Hits are added
// in ascending entry order = ascending index order within a row (fp32, multiply and add rounded
// separately, as Qdrant). on_row(row, score, any) runs once per row, in row order.
template <typename OnRow>
__device__ __forceinline__ void scan_rows(int64_t r0, int64_t r1, int lane, int32_t vocab,
                                          const int64_t* __restrict__ indptr,
                                          const int32_t* __restrict__ indices,
                                          const float* __restrict__ values,
                                          const int32_t* __restrict__ slot_of_term,
                                          const float* __restrict__ weights, int* lds_slot,
                                          float* lds_val, int* lds_pos, OnRow&& on_row) {
  if (r0 >= r1) return;
  const int64_t p_begin = indptr[r0];
  const int64_t p_end = indptr[r1];
  int64_t r = r0;
  int64_t win = r0;
  int64_t ends = (win + lane < r1) ? indptr[win + lane + 1] : p_end;
  int64_t e_cur = rl_64(ends, 0);
  float acc = 0.0f;
  bool any = false;
  auto next_row = [&]() {
    on_row(r, acc, any);
    acc = 0.0f;
    any = false;
    ++r;
    if (r < r1) {
      if (r - win >= 64) {
        win = r;
        ends = (win + lane < r1) ? indptr[win + lane + 1] : p_end;
      }
      e_cur = rl_64(ends, (int)(r - win));
    }
  };
  auto load_block = [&](int64_t p0, int32_t& t, float& v) {
    const int64_t j = p0 + lane;
    t = -1;
    v = 0.f;
    if (j < p_end) {
      t = indices[j];
      v = values[j];
    }
  };
  auto lookup = [&](int32_t t) -> int {
    int sl = -1;
    if (t >= 0 && t < vocab) sl = slot_of_term[t];
    return (sl >= 0 && sl < kSlots) ? sl : -1;
  };
  int32_t tb, tc;
  float va, vb, vc;
  load_block(p_begin, tb, va);
  int sa = lookup(tb);
  load_block(p_begin + 64, tb, vb);
  for (int64_t p0 = p_begin; p0 < p_end; p0 += 64) {
    const unsigned long long m = __ballot(sa >= 0);
    const int nh = __popcll(m);
    if (sa >= 0) {
      const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
      lds_slot[rank] = sa;
      lds_val[rank] = va;
      lds_pos[rank] = lane;
    }
    int sb = -1;
    bool prefetched = false;
    for (int h0 = 0; h0 < nh; h0 += kHitBatch) {
      float hw[kHitBatch];
#pragma unroll
      for (int u = 0; u < kHitBatch; ++u) {
        hw[u] = __uint_as_float(kAbsent);
        if (h0 + u < nh) hw[u] = weights[lds_slot[h0 + u] * kQB + lane];
      }
      if (!prefetched) {
        sb = lookup(tb);
        load_block(p0 + 128, tc, vc);
        prefetched = true;
      }
#pragma unroll
      for (int u = 0; u < kHitBatch; ++u) {
        if (h0 + u < nh) {
          const int64_t pos = p0 + __builtin_amdgcn_readfirstlane(lds_pos[h0 + u]);
          while (pos >= e_cur) next_row();
          if (__float_as_uint(hw[u]) != kAbsent) {
            acc = __fadd_rn(acc, __fmul_rn(hw[u], lds_val[h0 + u]));
            any = true;
          }
        }
      }
    }
    if (!prefetched) {
      sb = lookup(tb);
      load_block(p0 + 128, tc, vc);
    }
    sa = sb;
    va = vb;
    tb = tc;
    vb = vc;
  }
  while (r < r1) next_row();
}

__global__ __launch_bounds__(kScanThreads) void sparse_scan_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const float* __restrict__ values, const uint64_t* __restrict__ row_mask, int64_t n_rows,
    int64_t rows_per_wg, int nq, int32_t vocab, const int32_t* __restrict__ slot_of_term,
    const float* __restrict__ weights, const unsigned long long* __restrict__ qmask,
    float* __restrict__ cand_key, int32_t* __restrict__ cand_row, float* __restrict__ cand_bound) {
  __shared__ float lkey[kQB][kWavesPerWG * kLaneList];
  __shared__ int32_t lrow[kQB][kWavesPerWG * kLaneList];
  __shared__ float ldisc[kQB][kWavesPerWG];
  __shared__ int hslot[kWavesPerWG][64];
  __shared__ float hval[kWavesPerWG][64];
  __shared__ int hpos[kWavesPerWG][64];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int64_t lo = (int64_t)blockIdx.x * rows_per_wg;
  const int64_t hi = min(lo + rows_per_wg, n_rows);
  // contiguous rows per wave keep each wave's CSR stream sequential
  const int64_t span = hi > lo ? hi - lo : 0;
  const int64_t r0 = lo + span * wave / kWavesPerWG;
  const int64_t r1 = lo + span * (wave + 1) / kWavesPerWG;
  float s[kLaneList];
  int32_t ix[kLaneList];
#pragma unroll
  for (int j = 0; j < kLaneList; ++j) {
    s[j] = kNegInf;
    ix[j] = 0x7fffffff;
  }
  float disc = kNegInf;
  scan_rows(r0, r1, lane, vocab, indptr, indices, values, slot_of_term, weights, hslot[wave],
            hval[wave], hpos[wave], [&](int64_t row, float sc, bool hit) {
              if (row_mask && !((row_mask[row >> 6] >> (row & 63)) & 1ull)) return;
              if (__any(hit && sc > s[kLaneList - 1])) {
                if (hit) topm_insert(sc, (int32_t)row, s, ix, disc);
              } else if (hit) {
                disc = fmaxf(disc, sc);
              }
            });
#pragma unroll
  for (int j = 0; j < kLaneList; ++j) {
    lkey[lane][wave * kLaneList + j] = s[j];
    lrow[lane][wave * kLaneList + j] = ix[j];
  }
  ldisc[lane][wave] = disc;
  __syncthreads();
  // each wave merges 4 queries: 64 lane entries -> the best kKW, plus the bound
  for (int qq = 0; qq < kQB / kWavesPerWG; ++qq) {
    const int q = wave * (kQB / kWavesPerWG) + qq;
    if (q >= nq) break;
    float key = lkey[q][lane];
    int32_t row = lrow[q][lane];
    armi::wave_sort_approx_desc(key, row);
    const size_t base = (size_t)blockIdx.x * kQB + q;
    if (lane < kKW) {
      cand_key[base * kKW + lane] = key;
      cand_row[base * kKW + lane] = row;
    }
    float b = (lane < kWavesPerWG) ? ldisc[q][lane] : kNegInf;
    if (lane == kKW) b = fmaxf(b, key);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) b = fmaxf(b, __shfl_xor(b, off));
    if (lane == 0) cand_bound[base] = b;
  }
}

// One workgroup per query: keep the pooled entries >= t0 (the k-th largest workgroup maximum, a
// lower bound of the pooled k-th best), sort them, keep k, certify, emit.
__global__ __launch_bounds__(256) void sparse_merge_kernel(
    const float* __restrict__ cand_key, const int32_t* __restrict__ cand_row,
    const float* __restrict__ cand_bound, int n_wg, int q_first, int k, int64_t ordinal_base,
    float* __restrict__ out_scores, int64_t* __restrict__ out_ids,
    int32_t* __restrict__ out_count, uint32_t* __restrict__ flags, float* __restrict__ kth_out) {
  // flags / kth_out are indexed by the query's position within the pass (ql); outputs by qg
  __shared__ float skey[kSelCap];
  __shared__ int32_t srow[kSelCap];
  __shared__ float mx[256];
  __shared__ int32_t mxr[256];
  __shared__ float red[8];
  __shared__ int ctr[2];
  const int ql = blockIdx.x;
  const int qg = q_first + ql;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int pool = n_wg * kKW;
  float b = kNegInf;
  for (int g = tid; g < 256; g += 256) {
    float m = kNegInf;
    if (g < n_wg) {
      m = cand_key[((size_t)g * kQB + ql) * kKW];
      b = fmaxf(b, cand_bound[(size_t)g * kQB + ql]);
    }
    mx[g] = m;
    mxr[g] = g;
  }
  if (tid == 0) ctr[0] = 0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) b = fmaxf(b, __shfl_xor(b, off));
  if (lane == 0) red[wave] = b;
  armi::lds_sort_approx_desc(mx, mxr, 256);
  const float t0 = (n_wg >= k) ? mx[k - 1] : kNegInf;
  float dmax = kNegInf;
  for (int e = tid; e < pool; e += 256) {
    const size_t src = ((size_t)(e / kKW) * kQB + ql) * kKW + (e % kKW);
    const float kk = cand_key[src];
    if (kk == kNegInf) continue;
    if (kk >= t0) {
      const int slot = atomicAdd(&ctr[0], 1);
      if (slot < kSelCap) {
        skey[slot] = kk;
        srow[slot] = cand_row[src];
      }
    } else {
      dmax = fmaxf(dmax, kk);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) dmax = fmaxf(dmax, __shfl_xor(dmax, off));
  if (lane == 0) red[4 + wave] = dmax;
  __syncthreads();
  const int n_sel = ctr[0];
  const bool overflow = n_sel > kSelCap;
  const int n_keep = overflow ? kSelCap : n_sel;
  const int n2 = armi::pow2_at_least(max(n_keep, max(k, 2)));
  for (int e = n_keep + tid; e < n2; e += 256) {
    skey[e] = kNegInf;
    srow[e] = 0x7fffffff;
  }
  armi::lds_sort_approx_desc(skey, srow, n2);
  float bound = red[0];
#pragma unroll
  for (int w = 1; w < 8; ++w) bound = fmaxf(bound, red[w]);
  if (n2 > k) bound = fmaxf(bound, skey[k]);
  if (tid == 0) {
    int nv = 0;
    while (nv < n2 && nv < k && skey[nv] != kNegInf) ++nv;
    ctr[1] = nv;
  }
  __syncthreads();
  const int nv = ctr[1];
  bool certified;
  if (nv >= k)
    certified = skey[k - 1] > bound;
  else
    certified = (bound == kNegInf);
  certified = certified && !overflow;
  if (certified) {
    for (int c = tid; c < k; c += 256) {
      const size_t o = (size_t)qg * k + c;
      out_scores[o] = c < nv ? skey[c] : kNegInf;
      out_ids[o] = c < nv ? ordinal_base + srow[c] : -1;
    }
  }
  if (tid == 0) {
    out_count[qg] = certified ? nv : 0;
    flags[ql] |= certified ? ARMI_FLAG_CERTIFIED : 0u;
    // collection threshold of the fallback: the k-th candidate (a lower bound of the true k-th);
    // -inf when fewer than k candidates exist
    kth_out[ql] = certified ? std::numeric_limits<float>::infinity()
                            : (nv >= k ? skey[k - 1] : kNegInf);
  }
}

// Fallback scan: every row scoring >= thr[q] (and sharing an index) is appended to q's buffer.
__global__ __launch_bounds__(kScanThreads) void sparse_collect_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const float* __restrict__ values, const uint64_t* __restrict__ row_mask, int64_t n_rows,
    int64_t rows_per_wg, int nq, int32_t vocab, const int32_t* __restrict__ slot_of_term,
    const float* __restrict__ weights, const unsigned long long* __restrict__ qmask,
    const float* __restrict__ thr, int* __restrict__ coll_count, float* __restrict__ coll_key,
    int32_t* __restrict__ coll_row) {
  __shared__ int hslot[kWavesPerWG][64];
  __shared__ float hval[kWavesPerWG][64];
  __shared__ int hpos[kWavesPerWG][64];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const float t = lane < nq ? thr[lane] : std::numeric_limits<float>::infinity();
  if (__all(t == std::numeric_limits<float>::infinity())) return;
  const int64_t lo = (int64_t)blockIdx.x * rows_per_wg;
  const int64_t hi = min(lo + rows_per_wg, n_rows);
  const int64_t span = hi > lo ? hi - lo : 0;
  const int64_t r0 = lo + span * wave / kWavesPerWG;
  const int64_t r1 = lo + span * (wave + 1) / kWavesPerWG;
  scan_rows(r0, r1, lane, vocab, indptr, indices, values, slot_of_term, weights, hslot[wave],
            hval[wave], hpos[wave], [&](int64_t row, float sc, bool hit) {
              if (row_mask && !((row_mask[row >> 6] >> (row & 63)) & 1ull)) return;
              if (hit && sc >= t) {
                const int slot = atomicAdd(&coll_count[lane], 1);
                if (slot < kCollectCap) {
                  coll_key[(size_t)lane * kCollectCap + slot] = sc;
                  coll_row[(size_t)lane * kCollectCap + slot] = (int32_t)row;
                }
              }
            });
}

__global__ __launch_bounds__(256) void sparse_collect_merge_kernel(
    const int* __restrict__ coll_count, const float* __restrict__ coll_key,
    const int32_t* __restrict__ coll_row, int q_first, int k, int64_t ordinal_base,
    float* __restrict__ out_scores, int64_t* __restrict__ out_ids, int32_t* __restrict__ out_count,
    uint32_t* __restrict__ flags) {
  const int ql = blockIdx.x;
  const int qg = q_first + ql;
  if (flags[ql] & ARMI_FLAG_CERTIFIED) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* key = reinterpret_cast<float*>(smem);
  int32_t* row = reinterpret_cast<int32_t*>(smem + kCollectCap * 4);
  const int total = coll_count[ql];
  const int n = min(total, kCollectCap);
  const int n2 = armi::pow2_at_least(max(n, 2));
  for (int e = threadIdx.x; e < n2; e += 256) {
    key[e] = e < n ? coll_key[(size_t)ql * kCollectCap + e] : kNegInf;
    row[e] = e < n ? coll_row[(size_t)ql * kCollectCap + e] : 0x7fffffff;
  }
  armi::lds_sort_approx_desc(key, row, n2);
  const int nv = min(n, k);
  for (int c = threadIdx.x; c < k; c += 256) {
    const size_t o = (size_t)qg * k + c;
    out_scores[o] = c < nv ? key[c] : kNegInf;
    out_ids[o] = c < nv ? ordinal_base + row[c] : -1;
  }
  if (threadIdx.x == 0) {
    out_count[qg] = nv;
    flags[ql] |= ARMI_FLAG_FALLBACK | (total > kCollectCap ? kFlagOverflow : 0u);
  }
}

struct Plan {
  int n_wg;
  int64_t rows_per_wg;
  int pool2;
};

Plan plan(const armi_sparse_index* idx) {
  Plan p;
  const int64_t want = std::max<int64_t>(1, std::min<int64_t>(std::min(idx->num_cus, 256),
                                                              (idx->n_rows + 63) / 64));
  p.rows_per_wg = (idx->n_rows + want - 1) / want;
  if (p.rows_per_wg == 0) p.rows_per_wg = 1;
  p.n_wg = (int)((idx->n_rows + p.rows_per_wg - 1) / p.rows_per_wg);
  if (p.n_wg == 0) p.n_wg = 1;
  p.pool2 = 0;
  return p;
}

struct Workspace {
  int32_t* slot_of_term;
  float* weights;
  unsigned long long* qmask;
  float* cand_key;
  int32_t* cand_row;
  float* cand_bound;
  float* kth;
  int* coll_count;
  float* coll_key;
  int32_t* coll_row;
  size_t bytes;
};

Workspace carve(void* base, const armi_sparse_index* idx) {
  armi::Carver cv(base);
  Workspace w{};
  const Plan p = plan(idx);
  w.slot_of_term = cv.take<int32_t>((size_t)idx->vocab);
  w.weights = cv.take<float>((size_t)kQB * kMaxTerms * kQB);
  w.qmask = cv.take<unsigned long long>((size_t)kQB * kMaxTerms);
  w.cand_key = cv.take<float>((size_t)p.n_wg * kQB * kKW);
  w.cand_row = cv.take<int32_t>((size_t)p.n_wg * kQB * kKW);
  w.cand_bound = cv.take<float>((size_t)p.n_wg * kQB);
  w.kth = cv.take<float>(kQB);
  w.coll_count = cv.take<int>(kQB);
  w.coll_key = cv.take<float>((size_t)kQB * kCollectCap);
  w.coll_row = cv.take<int32_t>((size_t)kQB * kCollectCap);
  w.bytes = cv.off + 256;
  return w;
}

}  // namespace

extern "C" {

int armi_sparse_index_create(int device, const int64_t* indptr, const int32_t* indices,
                             const float* values, int64_t n_rows, int64_t nnz, int32_t vocab,
                             int64_t ordinal_base, armi_sparse_index** out, hipStream_t stream) {
  (void)stream;
  ARMI_REQUIRE(out != nullptr, "armi_sparse_index_create: out is null");
  *out = nullptr;
  ARMI_REQUIRE(n_rows >= 0 && n_rows < (int64_t(1) << 31), "armi_sparse_index_create: bad n_rows");
  ARMI_REQUIRE(vocab >= 1, "armi_sparse_index_create: vocab must be >= 1");
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
  idx->indptr = indptr;
  idx->indices = indices;
  idx->values = values;
  *out = idx;
  return ARMI_OK;
}

int armi_sparse_index_destroy(armi_sparse_index* index) {
  delete index;
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
  const Plan p = plan(idx);
  const size_t lds_collect = (size_t)kCollectCap * 8;
  ARMI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(sparse_collect_merge_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_collect));
  for (int q0 = 0; q0 < n_queries; q0 += kQB) {
    const int nqp = std::min(kQB, n_queries - q0);
    uint32_t* pflags = out_flags + q0;
    if (idx->n_rows == 0) {
      ARMI_HIP(hipMemsetAsync(out_count + q0, 0, sizeof(int32_t) * nqp, stream));
      ARMI_HIP(hipMemsetAsync(pflags, 0, sizeof(uint32_t) * nqp, stream));
      ARMI_HIP(hipMemsetAsync(out_ids + (size_t)q0 * k, 0xff, sizeof(int64_t) * nqp * k, stream));
      continue;
    }
    ARMI_HIP(hipMemsetAsync(w.slot_of_term, 0x7f, sizeof(int32_t) * idx->vocab, stream));
    ARMI_HIP(hipMemsetAsync(w.qmask, 0, sizeof(unsigned long long) * kQB * kMaxTerms, stream));
    ARMI_HIP(hipMemsetAsync(w.weights, 0xff, sizeof(float) * kQB * kMaxTerms * kQB, stream));
    ARMI_HIP(hipMemsetAsync(w.coll_count, 0, sizeof(int) * kQB, stream));
    term_slots_kernel<<<dim3(nqp), dim3(64), 0, stream>>>(q_indptr + q0, q_indices, idx->vocab,
                                                          w.slot_of_term);
    ARMI_LAUNCHED("term_slots_kernel");
    term_weights_kernel<<<dim3(nqp), dim3(64), 0, stream>>>(q_indptr + q0, q_indices, q_values,
                                                            idx->vocab, w.slot_of_term,
                                                            w.weights, w.qmask, pflags);
    ARMI_LAUNCHED("term_weights_kernel");
    sparse_scan_kernel<<<dim3(p.n_wg), dim3(kScanThreads), 0, stream>>>(
        idx->indptr, idx->indices, idx->values, row_mask, idx->n_rows, p.rows_per_wg, nqp,
        idx->vocab, w.slot_of_term, w.weights, w.qmask, w.cand_key, w.cand_row, w.cand_bound);
    ARMI_LAUNCHED("sparse_scan_kernel");
    sparse_merge_kernel<<<dim3(nqp), dim3(256), 0, stream>>>(
        w.cand_key, w.cand_row, w.cand_bound, p.n_wg, q0, k, idx->ordinal_base, out_scores,
        out_ids, out_count, pflags, w.kth);
    ARMI_LAUNCHED("sparse_merge_kernel");
    sparse_collect_kernel<<<dim3(p.n_wg), dim3(kScanThreads), 0, stream>>>(
        idx->indptr, idx->indices, idx->values, row_mask, idx->n_rows, p.rows_per_wg, nqp,
        idx->vocab, w.slot_of_term, w.weights, w.qmask, w.kth, w.coll_count, w.coll_key,
        w.coll_row);
    ARMI_LAUNCHED("sparse_collect_kernel");
    sparse_collect_merge_kernel<<<dim3(nqp), dim3(256), lds_collect, stream>>>(
        w.coll_count, w.coll_key, w.coll_row, q0, k, idx->ordinal_base, out_scores, out_ids,
        out_count, pflags);
    ARMI_LAUNCHED("sparse_collect_merge_kernel");
  }
  return ARMI_OK;
}

}  // extern "C"
