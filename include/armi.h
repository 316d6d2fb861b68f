/*
 * armi.h — C ABI of libarmi.so, the MI355X (gfx950) retrieval hot path of audio-rag.
 *
 * Each entry point replaces one piece of arithmetic that the reference delegates to a
 * third-party engine (all paths relative to the reference checkout):
 *
 *   armi_index_create / armi_index_destroy
 *       the Qdrant named vector "dense" = VectorParams(size=dim, distance=COSINE), filled by
 *       QdrantRetriever.add   src/audio_rag/retrieval/qdrant.py:93-109, 140-225
 *   armi_dense_topk
 *       Qdrant COSINE query_points(query=dense, using="dense", limit=k) and the dense
 *       Prefetch(limit=2*top_k) of hybrid search     src/audio_rag/retrieval/qdrant.py:284-288, 316-332
 *   armi_dense_exact_topk
 *       the same ranking computed by an exhaustive exact scan (fallback + test reference path)
 *   armi_sparse_*
 *       Qdrant sparse vector "sparse" (SparseVectorParams, no IDF modifier) and the sparse
 *       Prefetch / sparse query_points               src/audio_rag/retrieval/qdrant.py:103-107, 289-293, 299-312
 *   armi_rrf_fuse
 *       FusionQuery(fusion=Fusion.RRF)               src/audio_rag/retrieval/qdrant.py:295
 *   armi_topk_merge_shards
 *       the merge step that follows the RCCL all-gather of per-shard candidates (no reference
 *       counterpart: the reference runs one Qdrant replica, k8s/helm/audio-rag/values.yaml:137)
 *   armi_enc_*
 *       the non-GEMM ops of the XLM-RoBERTa cross-encoder behind CrossEncoder.predict
 *                                                    src/audio_rag/reranking/bge.py:119-123
 *
 * Conventions
 *   - Every function returns ARMI_OK (0) or a positive error code; the message of the last
 *     failure on the calling thread is returned by armi_last_error(). No C++ exception crosses
 *     this boundary.
 *   - Every array argument is caller-owned DEVICE memory unless the comment says "host".
 *   - Every launch is asynchronous and ordered on the given stream; nothing synchronises the
 *     host (graph capture safe). Workspaces are caller-allocated (see *_workspace_bytes).
 *   - An index is immutable after armi_index_create returns; any number of streams may search
 *     one index concurrently, each with its own workspace.
 *   - fp16 values are passed as their IEEE binary16 bit patterns (uint16_t).
 */
#ifndef ARMI_H
#define ARMI_H

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ARMI_OK 0
#define ARMI_ERR_INVALID 1     /* bad argument (shape, null pointer, unsupported size) */
#define ARMI_ERR_HIP 2         /* a HIP runtime call failed */
#define ARMI_ERR_UNSUPPORTED 3 /* valid request that this build does not implement */

/* ABI history. 1: rounds 1-3. 2 (round 5): armi_enc_cls_head_sigmoid takes the dense weight
 * transposed ([in][out], was [out][in]); armi_dense_topk_ex / _first / _second_pass,
 * armi_index_set_scan_cus and armi_cu_split_streams removed. A caller built against version 1
 * must not bind this library (armi_abi_version() tells). */
#define ARMI_ABI_VERSION 2

/* flags written per query by the top-k entry points */
#define ARMI_FLAG_CERTIFIED 1u /* fast path proved its top-k equal to the exact ranking */
#define ARMI_FLAG_FALLBACK 2u  /* fast path could not prove it; exact scan produced the answer */
#define ARMI_FLAG_FILTERED 4u  /* sparse: answered by the MFMA filter + exact rescore (with
                                * ARMI_FLAG_CERTIFIED) instead of the exact scan */

const char* armi_last_error(void);
int armi_abi_version(void);
/* sha256 prefix of the sources the library was built from (audio_rag_amd/_armi.py
 * source_digest); the Python loader refuses a library whose digest differs from csrc/. */
const char* armi_source_digest(void);

/* ------------------------------------------------------------------------------------------ */
/* Dense chunk store                                                                          */
/* ------------------------------------------------------------------------------------------ */

typedef struct armi_index armi_index;

/* rows: [n_rows][dim] fp16, row-major, caller-owned, must outlive the index.
 * Every component must be finite with |x| < 2 (BGE-M3 emits unit vectors); rows that violate
 * this are counted in armi_index_invalid_rows() and score as -inf.
 * dim must be 256, 512, 768 or 1024. ordinal_base is added to every row index to form
 * the chunk ordinal that the search functions return (corpus shards use base = first row). */
int armi_index_create(int device, const uint16_t* rows, int64_t n_rows, int dim,
                      int64_t ordinal_base, armi_index** out, hipStream_t stream);
int armi_index_destroy(armi_index* index);
int64_t armi_index_rows(const armi_index* index);
int armi_index_dim(const armi_index* index);
/* number of rows that failed validation (reads back a device counter: synchronises) */
int64_t armi_index_invalid_rows(const armi_index* index);
/* device pointers of the per-row norm arrays built at create time:
 *   norm2[r]     = sum_i (2^24 * x_ri)^2 as an exact int64
 *   inv_norm[r]  = 1.0 / sqrt((double) norm2[r])       (0.0 for a zero row)
 *   inv_norm32[r]= (float)(inv_norm[r] * 2^24)          (scale factor of the fast scan)
 * The index also keeps an int8 filter image of the rows (1 B per component, built at create
 * time: s_r = max_i |x_ri| / 127, round(x_ri / s_r)) with s_r / |x_r| and a Cauchy-Schwarz bound
 * of the quantisation error per row; the scans read it for k <= 64 (armi_dense_scan_form). */
int armi_index_norms(const armi_index* index, const int64_t** norm2, const double** inv_norm,
                     const float** inv_norm32);

/* The scan armi_dense_topk runs for n_queries queries and top-k (for roofline accounting):
 *   ARMI_SCAN_FP16         64-query scan over the fp16 rows (2 B per component)
 *   ARMI_SCAN_INT8_FILTER  64-query scan over the index's int8 filter image (1 B per component
 *                          + 8 B per row), then an exact fp16 rescore of the best upper bounds
 *                          (k <= 64; the default for those k)
 *   ARMI_SCAN_TILED_FP16   > 128 queries otherwise: the LDS-tiled MFMA scan over the fp16 rows
 *   ARMI_SCAN_TILED_INT8   > 128 queries, k <= 5, >= 200k rows: the LDS-tiled int8 x int8 MFMA
 *                          scan over the int8 image and per-call int8 queries (upper bounds),
 *                          then the exact fp16 rescore (the all-gathered batch of a multi-GPU
 *                          step over a large shard)
 * Results are the same exact ranking on every form. -1 for invalid arguments. */
#define ARMI_SCAN_FP16 0
#define ARMI_SCAN_INT8_FILTER 1
#define ARMI_SCAN_TILED_FP16 2
#define ARMI_SCAN_TILED_INT8 3
int armi_dense_scan_form(const armi_index* index, int n_queries, int k);

/* 1 when the call's ARMI_SCAN_INT8_FILTER passes stream the int8 image with nontemporal loads
 * (images larger than the Infinity Cache), else 0; -1 for invalid arguments. Introspection for
 * profiling (the kernel instance that runs); results do not depend on it. */
int armi_dense_scan_nontemporal(const armi_index* index, int n_queries, int k);

/* Workspace bytes needed by armi_dense_topk for n_queries queries and top-k. */
size_t armi_dense_workspace_bytes(const armi_index* index, int n_queries, int k);

/* Cosine top-k over the index.
 *   queries    [n_queries][dim] fp16 (same component rule as rows)
 *   k          1..240
 *   row_mask   nullable; bit r of the uint64 bitmask enables row r (metadata pre-filter)
 * outputs, each [n_queries][k]:
 *   out_scores  float cosine score (reference: hit.score, an fp32 dot of normalised vectors)
 *   out_ids     int64 chunk ordinal (ordinal_base + row); -1 past out_count
 *   out_rank    nullable double ranking key; the ranking is (key desc, ordinal asc)
 *   out_count   [n_queries] number of valid results (< k when fewer rows are enabled)
 *   out_flags   [n_queries] ARMI_FLAG_* bits
 * The result is the exact ranking of the fp16 inputs: key = (double)dot64 * inv_norm[row] where
 * dot64 = sum_i (2^24 q_i)(2^24 x_ri) is an exact int64 dot product. */
int armi_dense_topk(const armi_index* index, const uint16_t* queries, int n_queries, int k,
                    const uint64_t* row_mask, float* out_scores, int64_t* out_ids,
                    double* out_rank, int32_t* out_count, uint32_t* out_flags,
                    void* workspace, size_t workspace_bytes, hipStream_t stream);

size_t armi_dense_exact_workspace_bytes(const armi_index* index, int n_queries, int k);
/* Exhaustive exact scan with the same outputs and ranking as armi_dense_topk. */
int armi_dense_exact_topk(const armi_index* index, const uint16_t* queries, int n_queries, int k,
                          const uint64_t* row_mask, float* out_scores, int64_t* out_ids,
                          double* out_rank, int32_t* out_count, void* workspace,
                          size_t workspace_bytes, hipStream_t stream);

/* Merge per-shard top-k lists (after an all-gather) into the global top-k.
 *   in_*: [n_shards][n_queries][k_in], in_count [n_shards][n_queries]
 *   ranking (key desc, ordinal asc); outputs [n_queries][k_out] + out_count. */
int armi_topk_merge_shards(const double* in_rank, const float* in_scores, const int64_t* in_ids,
                           const int32_t* in_count, int n_shards, int n_queries, int k_in,
                           int k_out, double* out_rank, float* out_scores, int64_t* out_ids,
                           int32_t* out_count, hipStream_t stream);

/* armi_topk_merge_shards reading the all-gathered exchange buffer in place: per-shard lists
 * packed one (shard, query) row per byte row — the row of shard s and query q starts at
 * packed + s * shard_stride + q * query_stride (bytes) and holds k_in ranks (double) at
 * off_rank, k_in scores (float) at off_scores, k_in ids (int64) at off_ids and the count (int32)
 * at off_count. Fields must be naturally aligned and both strides multiples of 8. Saves the
 * per-field copies an unpacked call needs after the RCCL all-gather. */
int armi_topk_merge_shards_packed(const void* packed, int64_t shard_stride,
                                  int64_t query_stride, int64_t off_rank, int64_t off_scores,
                                  int64_t off_ids, int64_t off_count, int n_shards,
                                  int n_queries, int k_in, int k_out, double* out_rank,
                                  float* out_scores, int64_t* out_ids, int32_t* out_count,
                                  hipStream_t stream);

/* Live timing of the dominant kernels for roofline reporting (bench.py): while enabled, every
 * enable-th launch of a timed kernel (enable = 1: every launch; 0 disables) carries a HIP event
 * pair: a scan kernel's events are bound to its own dispatch (hipExtLaunchKernel: the kernel's
 * start and end, no marker packets), a whole sparse call is bracketed by events on its stream.
 * Launches under stream capture are not timed, and an armi_sparse_topk call whose whole stage is
 * timed does not also time its scan (period 2 alternates them). _read synchronises on the
 * recorded events of one slot, returns the summed time and the number of timed launches, and
 * clears them. Slots: ARMI_TIMING_DENSE_SCAN (the dense scan kernel of
 * armi_dense_topk), ARMI_TIMING_SPARSE_SCAN (the dominant scan of armi_sparse_topk: the MFMA
 * filter scan when the filter runs, else sparse_scan_kernel), ARMI_TIMING_ENCODER_GEMM (the
 * cross-encoder GEMMs of armi_enc_linear_f16), ARMI_TIMING_SPARSE_STAGE (a whole
 * armi_sparse_topk call).
 * armi_scan_timing_read = armi_kernel_timing_read(ARMI_TIMING_DENSE_SCAN, ...). */
#define ARMI_TIMING_DENSE_SCAN 0
#define ARMI_TIMING_SPARSE_SCAN 1
#define ARMI_TIMING_ENCODER_GEMM 2
#define ARMI_TIMING_SPARSE_STAGE 3  /* the whole armi_sparse_topk call (every pass, every kernel) */
#define ARMI_TIMING_SLOTS 4
int armi_scan_timing_enable(int enable);
int armi_scan_timing_read(double* total_ms, int64_t* launches);
int armi_kernel_timing_read(int slot, double* total_ms, int64_t* launches);

/* ------------------------------------------------------------------------------------------ */
/* Streaming query server (BASELINE configs[4] "streaming query at fixed QPS")                 */
/* ------------------------------------------------------------------------------------------ */
/* Replaces the reference's per-request search (src/audio_rag/api/v1/query.py:90-115 calling
 * QdrantRetriever.search, src/audio_rag/retrieval/qdrant.py:227-352, one query per request):
 * single dense queries submitted from any thread are coalesced into batches of up to max_batch
 * (a batch leaves when full or max_wait_us after its first query) and answered by
 * armi_dense_topk on the server's own HIP stream, with up to three batches in flight. Results are
 * those of armi_dense_topk for that query alone (exact ranking). Thread-safe; the index must
 * outlive the server. */
typedef struct armi_stream armi_stream;
typedef struct armi_sparse_index armi_sparse_index; /* declared again below */
int armi_stream_create(const armi_index* index, int k, int max_batch, double max_wait_us,
                       armi_stream** out);
/* Hybrid server: a query submitted with sparse terms is answered as QdrantRetriever.search's
 * hybrid branch (qdrant.py:272-298: dense and sparse prefetch 2k, armi_rrf_fuse with rrf_k,
 * limit k; scores are the RRF scores, in `rank` as fp64); one submitted without terms as its
 * dense branch (dense top-k, cosine scores). k <= 120. Both indexes must outlive the server. */
int armi_stream_create_hybrid(const armi_index* index, const armi_sparse_index* sparse, int k,
                              int rrf_k, int max_batch, double max_wait_us, armi_stream** out);
/* Stops the server (no new batches; blocked submitters and waiters wake and return an error);
 * the server stays allocated until armi_stream_destroy. */
int armi_stream_stop(armi_stream* server);
/* Stops the server, waits for every caller still inside submit / wait / stats / loadgen to
 * return, then frees it. */
int armi_stream_destroy(armi_stream* server);
/* query: host fp16 [dim], copied before return; *ticket identifies its result. */
int armi_stream_submit(armi_stream* server, const uint16_t* query, int64_t* ticket);
/* The same with the query's sparse terms (ascending indices, nnz <= 256; nnz = 0 = no sparse
 * vector); needs a hybrid server when nnz > 0. */
int armi_stream_submit_hybrid(armi_stream* server, const uint16_t* query,
                              const int32_t* sp_indices, const float* sp_values, int nnz,
                              int64_t* ticket);
/* Branch and filter per query (QdrantRetriever.search's choice, qdrant.py:262-332):
 * a query "carries a sparse vector" when sp_indices and sp_values are both non-null, even with
 * nnz = 0 (the reference's `if query.sparse` is true for an empty SparseVector object).
 * mode ARMI_STREAM_AUTO = hybrid when the query carries a sparse vector (hybrid server), else
 * dense; ARMI_STREAM_DENSE = the dense branch whatever the terms; ARMI_STREAM_SPARSE =
 * sparse-only (top-k of the sparse dot, hit.score = that dot) when the query carries a sparse
 * vector, else dense (the reference's fallback). An empty sparse vector gives RRF over the dense
 * list alone (hybrid) or an empty result (sparse-only). Sparse terms need a hybrid server. row_mask (nullable) = a device
 * bitmask over the store's ordinals (armi_dense_topk's row_mask: the Qdrant payload filter),
 * caller-owned, unchanged and alive until the ticket's wait has returned; it applies to every
 * list of the query (dense, sparse, both prefetches). A batch holds queries of one row_mask: a
 * query with another mask closes the collecting batch (it leaves at once) and opens the next. */
#define ARMI_STREAM_AUTO 0
#define ARMI_STREAM_DENSE 1
#define ARMI_STREAM_SPARSE 2
int armi_stream_submit_ex(armi_stream* server, const uint16_t* query, const int32_t* sp_indices,
                          const float* sp_values, int nnz, int mode, const uint64_t* row_mask,
                          int64_t* ticket);
/* Blocks until the ticket's result is published (at most timeout_us), then copies its k
 * scores / ids / rank keys (each nullable), the valid count and the branch taken (mode:
 * 0 dense, 1 hybrid, 2 sparse-only; nullable). Results stay readable until R later tickets have been
 * published, R = the largest power of two whose ring (R (k (4 + 8 + 8) + 48) B of host memory)
 * fits 128 MiB, at least max(2^14, 64 max_batch): 2^19 tickets at k = 10. An older ticket fails
 * with "result overwritten"; the copy is re-validated after it is taken, so a caller never
 * receives another ticket's results. */
int armi_stream_wait(armi_stream* server, int64_t ticket, float* scores, int64_t* ids,
                     double* rank, int32_t* count, int32_t* mode, double timeout_us);
int armi_stream_stats(armi_stream* server, int64_t* batches, int64_t* queries);
/* Native open-loop load generator (bench.py --workload stream): n_queries arrivals as a
 * Poisson process at `qps` from one thread, query i = row (i % n_vectors) of `queries` (host
 * fp16 [n_vectors][dim]) with, when q_indptr is non-null, the sparse terms of CSR row
 * (i % n_vectors); latency_us[i] = completion - submit of query i; elapsed_s = last
 * completion - first submit. Results are collected by a second thread while arrivals continue,
 * so n_queries is unbounded; out_ids [n_queries][k] / out_count [n_queries] (nullable) receive
 * every query's answer (ids of the branch taken, as armi_stream_wait). */
int armi_stream_loadgen(armi_stream* server, const uint16_t* queries, const int32_t* q_indptr,
                        const int32_t* q_indices, const float* q_values, int64_t n_vectors,
                        int64_t n_queries, double qps, uint64_t seed, double* latency_us,
                        double* elapsed_s, int64_t* completed, int64_t* out_ids,
                        int32_t* out_count);

/* ------------------------------------------------------------------------------------------ */
/* Sparse (lexical-weight) store                                                              */
/* ------------------------------------------------------------------------------------------ */

typedef struct armi_sparse_index armi_sparse_index;

/* CSR corpus: indptr [n_rows+1] int64, indices [nnz] int32 (strictly ascending per row),
 * values [nnz] float. Caller-owned, must outlive the index. */
int armi_sparse_index_create(int device, const int64_t* indptr, const int32_t* indices,
                             const float* values, int64_t n_rows, int64_t nnz, int32_t vocab,
                             int64_t ordinal_base, armi_sparse_index** out, hipStream_t stream);
int armi_sparse_index_destroy(armi_sparse_index* index);

size_t armi_sparse_workspace_bytes(const armi_sparse_index* index, int n_queries, int k);
/* Sparse dot-product top-k. Query CSR: q_indptr [n_queries+1] int32 (absolute offsets),
 * q_indices ascending int32 (at most 256 per query: a longer query is scored on its first 256
 * terms and gets flag bit 8; the Python layer refuses such queries before the call), q_values float.
 * out_flags: ARMI_FLAG_CERTIFIED (merged lists proved exact) or ARMI_FLAG_FALLBACK (answer from
 * the collecting rescan, or, when more than 4096 rows reach its threshold, from an exact
 * term-at-a-time rescoring of the shard by helper workgroups: exact either way). score = sum
 * over shared indices, ascending index order, of fl32(q*d) accumulated in fp32 (mul and add
 * rounded separately). Only rows that share at least one index with the query are results.
 * Ranking (score desc, ordinal asc).
 * When every value of the index is >= 0 and k <= 128, a pass of at most 512 distinct terms is
 * first answered by the MFMA filter (upper bounds of every row's score from u8 levels on the
 * matrix cores, exact rescore of the best candidates, certificate): such
 * queries get ARMI_FLAG_CERTIFIED | ARMI_FLAG_FILTERED; the exact scan answers the rest. The
 * results are the same either way. */
int armi_sparse_topk(const armi_sparse_index* index, const int32_t* q_indptr,
                     const int32_t* q_indices, const float* q_values, int n_queries, int k,
                     const uint64_t* row_mask, float* out_scores, int64_t* out_ids,
                     int32_t* out_count, uint32_t* out_flags, void* workspace,
                     size_t workspace_bytes, hipStream_t stream);

/* Enables (1) or disables (0) the MFMA filter of armi_sparse_topk on this index (default on:
 * the exact scan alone when off); usable (host, nullable) = 1 when the index can use the filter
 * (every value >= 0), else 0. No search may be in flight on the index. */
int armi_sparse_index_set_filter(armi_sparse_index* index, int enable, int* usable);

/* Query-term exchange of the sharded hybrid step (retrieval/shards.py; no reference
 * counterpart, the reference queries one Qdrant replica). _pack: CSR -> fixed slots (count
 * int32 [n], slot_indices int32 [n][slots], slot_values float [n][slots], zero-filled; terms past
 * `slots` are dropped, so callers refuse longer queries first). _unpack: the all-gathered rows
 * (row q at rows + q * row_stride, its count / indices / values at the byte offsets) -> CSR
 * (indptr int32 [n + 1], indices, values; capacity n * slots), read in place. */
int armi_query_slots_pack(const int32_t* indptr, const int32_t* indices, const float* values,
                          int n_queries, int slots, int32_t* count, int32_t* slot_indices,
                          float* slot_values, hipStream_t stream);
int armi_query_slots_unpack(const void* rows, int64_t row_stride, int64_t off_count,
                            int64_t off_indices, int64_t off_values, int n_queries, int slots,
                            int32_t* indptr, int32_t* indices, float* values,
                            hipStream_t stream);

/* ------------------------------------------------------------------------------------------ */
/* Reciprocal-rank fusion                                                                     */
/* ------------------------------------------------------------------------------------------ */

/* For each query: score[id] = sum over the two lists of 1/(rrf_k + pos) (pos 0-based, fp64,
 * list a added first), sorted by score descending; ties keep first-seen order (all of list a in
 * order, then the ids only in list b in order). Lists hold ka / kb slots per query, of which
 * a_count / b_count are valid. Outputs [n_queries][limit] + out_count. */
int armi_rrf_fuse(const int64_t* a_ids, const int32_t* a_count, int ka, const int64_t* b_ids,
                  const int32_t* b_count, int kb, int n_queries, int rrf_k, int limit,
                  int64_t* out_ids, double* out_scores, int32_t* out_count, hipStream_t stream);

/* ------------------------------------------------------------------------------------------ */
/* Cross-encoder (XLM-RoBERTa) non-GEMM ops; all activations fp32 row-major                    */
/* ------------------------------------------------------------------------------------------ */

/* out[t] = LayerNorm(x[t] + res[t]) * gamma + beta over the last dim (res nullable). */
int armi_enc_layernorm_residual(const float* x, const float* res, const float* gamma,
                                const float* beta, float* out, int64_t n_rows, int width,
                                float eps, hipStream_t stream);
/* in-place softmax over the last dim of scores [n_seq][heads][L][L] scaled by `scale`,
 * keys with mask[seq][key] == 0 excluded. */
int armi_enc_masked_softmax(float* scores, const int32_t* mask, int n_seq, int heads, int L,
                            float scale, hipStream_t stream);
/* in-place exact (erf) GELU of x + bias[col]; bias nullable. */
int armi_enc_bias_gelu(float* x, const float* bias, int64_t n_rows, int width,
                       hipStream_t stream);
/* XLM-R embeddings: word[ids] + pos[padding_idx + cumsum(ids != pad)] + type[0], then
 * LayerNorm. ids [n_seq][L] int32; word [vocab][width], pos [n_pos][width]. Ids outside
 * [0, vocab) embed as <unk> (id 3) and positions are clamped to n_pos - 1, so no input can read
 * outside the tables. */
int armi_enc_embed(const int32_t* ids, const float* word, const float* pos, const float* type0,
                   const float* gamma, const float* beta, float* out, int n_seq, int L,
                   int width, int pad_id, int vocab, int n_pos, float eps, hipStream_t stream);
/* The same over fp16 tables (the fp16 model's own word / position / type embeddings, no fp32
 * copy: BGE-M3's word table is 0.5 GB in fp16), writing the fp16 activations the fp16 forwards
 * feed their first GEMM: out [n_seq][L][width] fp16, the round-to-nearest-even of a LayerNorm
 * computed in fp32 from the same (fp16-exact) table values. Equal to armi_enc_embed's output up
 * to the fp32 rounding of the LayerNorm statistics, not bitwise: the width % 256 == 0 path
 * (one workgroup per 32-token chunk) sums a row's components in a different order. */
int armi_enc_embed_f16(const int32_t* ids, const uint16_t* word, const uint16_t* pos,
                       const uint16_t* type0, const float* gamma, const float* beta, uint16_t* out,
                       int n_seq, int L, int width, int pad_id, int vocab, int n_pos, float eps,
                       hipStream_t stream);
/* classification head on token 0: sigmoid(out_w . tanh(dense_w h0 + dense_b) + out_b)
 * hidden [n_seq][L][width] -> out [n_seq]; dense_wt = dense_w transposed, [width_in][width_out]
 * row-major (nn.Linear's weight.t()); width a multiple of 4, <= 1024 (8 sequences per
 * workgroup, one thread per output feature). */
int armi_enc_cls_head_sigmoid(const float* hidden, const float* dense_wt, const float* dense_b,
                              const float* out_w, const float* out_b, float* out, int n_seq,
                              int L, int width, hipStream_t stream);

/* fp16 forward pieces (fp16 GEMM operands, fp32 residual stream / statistics).
 * Fused masked self-attention of XLMRobertaSelfAttention (eager QK^T -> softmax -> PV of
 * transformers, as CrossEncoder.predict runs it for BGEReranker, reranking/bge.py:119-123):
 *   qkv  [n_seq][L][3][heads][head_dim] fp16 (the fused Q|K|V projection output)
 *   mask [n_seq][L] int32 key mask (0 = padding key)
 *   ctx  [n_seq][L][heads][head_dim] fp16 = softmax(Q K^T * scale + mask) V
 * head_dim must be 64, L <= 512. Scores and softmax statistics are fp32; P is rounded to fp16
 * for the P.V product (fp32 accumulate). */
int armi_enc_attention_f16(const uint16_t* qkv, const int32_t* mask, uint16_t* ctx, int n_seq,
                           int L, int heads, int head_dim, float scale, hipStream_t stream);
/* Attention of the <s> query (position 0) of each sequence over its keys, same qkv / mask
 * layout as armi_enc_attention_f16; ctx is [n_seq][heads][head_dim] fp16. The last layer of the
 * cross-encoder only feeds the classification head's <s> row (CrossEncoder.predict ->
 * XLMRobertaClassificationHead, reranking/bge.py:119-123), so only that query row is computed.
 * Scores, softmax and the P.V sum are fp32. */
int armi_enc_attention_cls_f16(const uint16_t* qkv, const int32_t* mask, uint16_t* ctx,
                               int n_seq, int L, int heads, int head_dim, float scale,
                               hipStream_t stream);
/* out = LayerNorm(x + res) with x fp16 and res fp32 (nullable); writes fp32 out and, when out16
 * is not null, its fp16 rounding (the next GEMM's operand). */
int armi_enc_layernorm_residual_f16(const uint16_t* x, const float* res, const float* gamma,
                                    const float* beta, float* out, uint16_t* out16,
                                    int64_t n_rows, int width, float eps, hipStream_t stream);
/* out16 = LayerNorm(x + res) with fp16 x, res and output (fp32 statistics): the all-fp16
 * residual stream of the default fp16 cross-encoder forward. width must be 768 or 1024. */
int armi_enc_add_layernorm_f16(const uint16_t* x, const uint16_t* res, const float* gamma,
                               const float* beta, uint16_t* out16, int64_t n_rows, int width,
                               float eps, hipStream_t stream);
/* in-place exact (erf) GELU of fp16 x (+ fp32 bias[col], nullable), computed in fp32;
 * width must be a multiple of 8. */
int armi_enc_gelu_f16(uint16_t* x, const float* bias, int64_t n_rows, int width,
                      hipStream_t stream);
/* out = epi(x . w^T + bias): the nn.Linear layers of the cross-encoder (XLMRobertaLayer as
 * CrossEncoder.predict runs it, reranking/bge.py:119-123) on the hand-written gfx950 MFMA GEMM,
 * with the intermediate dense's exact-erf GELU (XLMRobertaIntermediate) fused into the epilogue.
 *   x [m][k] fp16, w [n][k] fp16 (nn.Linear weight layout), bias [n] fp32, out [m][n] fp16;
 *   fp32 accumulate; n % 256 == 0, k % 64 == 0, k <= 8192.
 * Timed under ARMI_TIMING_ENCODER_GEMM when live timing is on. */
#define ARMI_EPI_BIAS 0
#define ARMI_EPI_BIAS_GELU 1
int armi_enc_linear_f16(const uint16_t* x, const uint16_t* w, const float* bias, uint16_t* out,
                        int64_t m, int n, int k, int epilogue, hipStream_t stream);
/* The same layer for the query encodes of BGE-M3 (embeddings/bge.py:137-157 through
 * embeddings/xlmr_f16.py): a weight stream, 16 output columns x 32 token rows per workgroup, K
 * split over its 8 (16 for k = 3072 / 4096) waves and summed in a fixed order. A row's result
 * depends only on its own inputs and k, not on m: a query encoded alone and inside a batch gets
 * the same bits. m <= 32 * 65535, n % 16 == 0, k % 256 == 0; bias fp32 [n]. */
int armi_enc_linear_small_f16(const uint16_t* x, const uint16_t* w, const float* bias,
                              uint16_t* out, int m, int n, int k, int epilogue,
                              hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* ARMI_H */
