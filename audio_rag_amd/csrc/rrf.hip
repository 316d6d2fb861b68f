// Reciprocal-rank fusion of the dense and sparse prefetch lists (gfx950).
//
// Restates FusionQuery(fusion=Fusion.RRF) as issued by QdrantRetriever.search
// (src/audio_rag/retrieval/qdrant.py:281-298) with the semantics of qdrant-client's local-mode
// reciprocal_rank_fusion (qdrant-client >= 1.14.3, pyproject.toml:25, not vendored):
//   score[id] = sum over prefetch lists of 1 / (2 + pos), pos 0-based, summed in fp64 in list
//   order (dense list first); results sorted by score descending with a stable sort, so equal
//   scores keep first-seen order (dense-list ids in dense order, then sparse-only ids).
// One wave per query; both lists hold ids unique within the list (they come from top-k).
#include <limits>

#include "armi_common.h"

namespace {

constexpr int kMaxList = 256;
constexpr int kPool = 2 * kMaxList;  // power of two

__global__ __launch_bounds__(64) void rrf_kernel(const int64_t* __restrict__ a_ids,
                                                 const int32_t* __restrict__ a_count, int ka,
                                                 const int64_t* __restrict__ b_ids,
                                                 const int32_t* __restrict__ b_count, int kb,
                                                 int rrf_k, int limit,
                                                 int64_t* __restrict__ out_ids,
                                                 double* __restrict__ out_scores,
                                                 int32_t* __restrict__ out_count) {
  __shared__ double score[kPool];
  __shared__ int64_t id[kPool];
  __shared__ int32_t seen[kPool];
  __shared__ int32_t b_match[kMaxList];
  const int q = blockIdx.x;
  const int lane = threadIdx.x;
  const int ca = min(max(a_count[q], 0), ka);
  const int cb = min(max(b_count[q], 0), kb);
  const int64_t* a = a_ids + (size_t)q * ka;
  const int64_t* b = b_ids + (size_t)q * kb;

  // sort only the power of two covering both lists
  const int n2 = armi::pow2_at_least(max(ca + cb, 2));
  for (int i = lane; i < n2; i += 64) {
    score[i] = -std::numeric_limits<double>::infinity();
    id[i] = -1;
    seen[i] = 0x7fffffff;
  }
  __syncthreads();
  for (int i = lane; i < ca; i += 64) {
    id[i] = a[i];
    score[i] = 1.0 / (double)(rrf_k + i);
    seen[i] = i;
  }
  __syncthreads();
  // each sparse id: its slot in the dense list, or -1
  for (int j = lane; j < cb; j += 64) {
    const int64_t x = b[j];
    int hit = -1;
    for (int i = 0; i < ca; ++i)
      if (id[i] == x) { hit = i; break; }
    b_match[j] = hit;
  }
  __syncthreads();
  // matched: add in the dense-then-sparse order of the reference; unmatched: append in order
  int appended = 0;
  for (int j0 = 0; j0 < cb; j0 += 64) {
    const int j = j0 + lane;
    const bool valid = j < cb;
    const int hit = valid ? b_match[j] : -2;
    if (hit >= 0) score[hit] = score[hit] + 1.0 / (double)(rrf_k + j);
    const bool fresh = (hit == -1);
    const unsigned long long m = __ballot(fresh);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (fresh) {
      const int slot = ca + appended + before;
      id[slot] = b[j];
      score[slot] = 1.0 / (double)(rrf_k + j);
      seen[slot] = slot;
    }
    appended += __popcll(m);
  }
  const int n = ca + appended;
  __syncthreads();
  // stable descending sort: key (score desc, seen asc)
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = lane; t < n2 / 2; t += 64) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const bool hi_better =
            score[hi] > score[lo] || (score[hi] == score[lo] && seen[hi] < seen[lo]);
        if (hi_better == desc) {
          const double ts = score[lo]; score[lo] = score[hi]; score[hi] = ts;
          const int64_t ti = id[lo]; id[lo] = id[hi]; id[hi] = ti;
          const int32_t tn = seen[lo]; seen[lo] = seen[hi]; seen[hi] = tn;
        }
      }
      __syncthreads();
    }
  }
  const int n_out = min(n, limit);
  for (int c = lane; c < limit; c += 64) {
    const size_t o = (size_t)q * limit + c;
    out_ids[o] = c < n_out ? id[c] : -1;
    out_scores[o] = c < n_out ? score[c] : 0.0;
  }
  if (lane == 0) out_count[q] = n_out;
}

}  // namespace

extern "C" int armi_rrf_fuse(const int64_t* a_ids, const int32_t* a_count, int ka,
                             const int64_t* b_ids, const int32_t* b_count, int kb, int n_queries,
                             int rrf_k, int limit, int64_t* out_ids, double* out_scores,
                             int32_t* out_count, hipStream_t stream) {
  ARMI_REQUIRE(ka >= 1 && ka <= kMaxList && kb >= 1 && kb <= kMaxList,
               "armi_rrf_fuse: list widths must be in [1, 256]");
  ARMI_REQUIRE(limit >= 1, "armi_rrf_fuse: limit must be >= 1");
  ARMI_REQUIRE(rrf_k >= 1, "armi_rrf_fuse: rrf_k must be >= 1 (1/(rrf_k + pos) at pos 0)");
  if (n_queries <= 0) return ARMI_OK;
  ARMI_REQUIRE(a_ids && a_count && b_ids && b_count && out_ids && out_scores && out_count,
               "armi_rrf_fuse: null pointer argument");
  rrf_kernel<<<dim3(n_queries), dim3(64), 0, stream>>>(a_ids, a_count, ka, b_ids, b_count, kb,
                                                       rrf_k, limit, out_ids, out_scores,
                                                       out_count);
  ARMI_LAUNCHED("rrf_kernel");
  return ARMI_OK;
}
