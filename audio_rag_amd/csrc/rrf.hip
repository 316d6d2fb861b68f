// Reciprocal-rank fusion of the dense and sparse prefetch lists (gfx950).
//
// Restates FusionQuery(fusion=Fusion.RRF) as issued by QdrantRetriever.search
// (src/audio_rag/retrieval/qdrant.py:281-298) with the semantics of qdrant-client's local-mode
// reciprocal_rank_fusion (qdrant-client >= 1.14.3, pyproject.toml:25, not vendored):
//   score[id] = sum over prefetch lists of 1 / (2 + pos), pos 0-based, summed in fp64 in list
//   order (dense list first); results sorted by score descending with a stable sort, so equal
//   scores keep first-seen order (dense-list ids in dense order, then sparse-only ids).
// One wave per query; both lists hold ids unique within the list (they come from top-k). The
// fused order is found by counting (each slot's rank = slots ahead of it), not by a sort.
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
  __shared__ int64_t a_lds[kMaxList];
  __shared__ int32_t b_match[kMaxList];
  const int q = blockIdx.x;
  const int lane = threadIdx.x;
  const int ca = min(max(a_count[q], 0), ka);
  const int cb = min(max(b_count[q], 0), kb);
  const int64_t* a = a_ids + (size_t)q * ka;
  const int64_t* b = b_ids + (size_t)q * kb;

  // slot s of the pool = first-seen position: dense ids in dense order, then the sparse-only ids
  // in sparse order (the reference's dict insertion order); its ranking key is (score desc, s asc)
  for (int i = lane; i < ca; i += 64) {
    const int64_t x = a[i];
    a_lds[i] = x;
    id[i] = x;
    score[i] = 1.0 / (double)(rrf_k + i);
  }
  __syncthreads();
  // each sparse id: its slot in the dense list, or -1 (the dense ids are read as LDS broadcasts)
  for (int j = lane; j < cb; j += 64) {
    const int64_t x = b[j];
    int hit = -1;
    for (int i = ca - 1; i >= 0; --i) hit = a_lds[i] == x ? i : hit;
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
    }
    appended += __popcll(m);
  }
  const int n = ca + appended;
  __syncthreads();
  // rank by counting: the final position of slot p is the number of slots ranked ahead of it
  // (higher score, or equal score and earlier slot: the stable descending sort); every lane
  // reads the pool as LDS broadcasts, no sorting network and no barrier per stage
  const int n_out = min(n, limit);
  for (int p = lane; p < n; p += 64) {
    const double sp = score[p];
    int r = 0;
    for (int o = 0; o < n; ++o) {
      const double so = score[o];
      r += (so > sp || (so == sp && o < p)) ? 1 : 0;
    }
    if (r < n_out) {
      const size_t dst = (size_t)q * limit + r;
      out_ids[dst] = id[p];
      out_scores[dst] = sp;
    }
  }
  for (int c = n_out + lane; c < limit; c += 64) {
    const size_t dst = (size_t)q * limit + c;
    out_ids[dst] = -1;
    out_scores[dst] = 0.0;
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
