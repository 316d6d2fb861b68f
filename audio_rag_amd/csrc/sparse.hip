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

// Score one row for this lane's query. Returns false when the row shares no index with it.
__device__ __forceinline__ bool score_row(int64_t a, int64_t e, int lane, int32_t vocab,
                                          const int32_t* __restrict__ indices,
                                          const float* __restrict__ values,
                                          const int32_t* __restrict__ slot_of_term,
                                          const float* __restrict__ weights,
                                          const unsigned long long* __restrict__ qmask,
                                          float& score) {
  float acc = 0.0f;
  bool any = false;
  for (int64_t c0 = a; c0 < e; c0 += 64) {
    const int64_t j = c0 + lane;
    int s = kNoSlot;
    float dv = 0.f;
    if (j < e) {
      const int32_t t = indices[j];
      if (t >= 0 && t < vocab) s = slot_of_term[t];
      dv = values[j];
    }
    // a slot is a pair index of this pass: anything else (the memset pattern) is "absent"
    const bool present = s >= 0 && s < kQB * kMaxTerms;
    unsigned long long m = __ballot(present);
    while (m) {
      // up to 8 hits in flight, then accumulate them in ascending index order
      int hs[8];
      float hv[8], hw[8];
      unsigned long long hq[8];
      int nh = 0;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (m) {
          const int b = __ffsll((long long)m) - 1;
          m &= m - 1;
          hs[u] = __shfl(s, b);
          hv[u] = __shfl(dv, b);
          nh = u + 1;
        } else {
          hs[u] = 0;
          hv[u] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (u < nh) {
          hq[u] = qmask[hs[u]];
          hw[u] = weights[(size_t)hs[u] * kQB + lane];
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (u < nh && ((hq[u] >> lane) & 1ull)) {
          acc = __fadd_rn(acc, __fmul_rn(hw[u], hv[u]));
          any = true;
        }
      }
    }
  }
  score = acc;
  return any;
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
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int64_t lo = (int64_t)blockIdx.x * rows_per_wg;
  const int64_t hi = min(lo + rows_per_wg, n_rows);
  float s[kLaneList];
  int32_t ix[kLaneList];
#pragma unroll
  for (int j = 0; j < kLaneList; ++j) {
    s[j] = kNegInf;
    ix[j] = 0x7fffffff;
  }
  float disc = kNegInf;
  for (int64_t r = lo + wave; r < hi; r += kWavesPerWG) {
    if (row_mask && !((row_mask[r >> 6] >> (r & 63)) & 1ull)) continue;
    float sc;
    const bool hit = score_row(indptr[r], indptr[r + 1], lane, vocab, indices, values,
                               slot_of_term, weights, qmask, sc);
    if (__any(hit && sc > s[kLaneList - 1]) ) {
      if (hit) topm_insert(sc, (int32_t)r, s, ix, disc);
    } else if (hit) {
      disc = fmaxf(disc, sc);
    }
  }
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
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const float t = lane < nq ? thr[lane] : std::numeric_limits<float>::infinity();
  if (__all(t == std::numeric_limits<float>::infinity())) return;
  const int64_t lo = (int64_t)blockIdx.x * rows_per_wg;
  const int64_t hi = min(lo + rows_per_wg, n_rows);
  for (int64_t r = lo + wave; r < hi; r += kWavesPerWG) {
    if (row_mask && !((row_mask[r >> 6] >> (r & 63)) & 1ull)) continue;
    float sc;
    const bool hit = score_row(indptr[r], indptr[r + 1], lane, vocab, indices, values,
                               slot_of_term, weights, qmask, sc);
    if (hit && sc >= t) {
      const int slot = atomicAdd(&coll_count[lane], 1);
      if (slot < kCollectCap) {
        coll_key[(size_t)lane * kCollectCap + slot] = sc;
        coll_row[(size_t)lane * kCollectCap + slot] = (int32_t)r;
      }
    }
  }
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
