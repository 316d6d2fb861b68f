// Native streaming query server (BASELINE configs[4] "streaming query at fixed QPS"): single
// dense queries from any number of caller threads coalesced into device batches.
//
// The reference answers one request at a time: the REST route calls pipeline.query() per
// request (src/audio_rag/api/v1/query.py:90-115) in each of 4 uvicorn processes
// (Dockerfile.api:85-86), so Qdrant sees batch-1 searches. On the MI355X a batch-1 scan costs the
// same HBM pass over the chunk store as a batch-64 scan, so the serving layer batches across
// requests. This is that layer without an interpreter in the request path:
//   submit (any thread): copy the query into the collecting batch (pinned host memory), take a
//     ticket; the first query of a batch starts its max_wait clock.
//   dispatcher thread: when the batch is full or its first query has waited max_wait, hand it
//     to one of kSlots in-flight slots: H2D copy, armi_dense_topk, D2H copy of the results, an
//     event -- all on the server's HIP stream -- and start collecting the next batch while the
//     GPU runs (slots recycle in order).
//   completion thread: per slot in order, wait for its event, copy every query's top-k into the
//     result ring, stamp the completion time, wake the waiters.
//   wait (caller): block until its ticket's ring entry is complete, copy the results out.
// Per-query semantics are armi_dense_topk's (exact cosine ranking, certified fast scan, exact
// fallback inside the call); only the grouping is new. A hybrid server (armi_stream_create_hybrid)
// answers each query as QdrantRetriever.search's hybrid branch does (qdrant.py:272-298): dense and
// sparse prefetches of 2k, RRF 1/(rrf_k + pos) with the dense list first, limit k; a query
// submitted without sparse terms takes the dense branch (qdrant.py:316-323: its dense top-k).
// armi_stream_submit_ex adds the sparse-only branch (qdrant.py:299-311: the first k of the
// batch's sparse top-2k list, which is the sparse top-k: one ranking, (score desc, id asc)) and
// the payload filter (a device row bitmask per batch: a query with another mask seals the
// collecting batch, which the dispatcher then hands over at once).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "armi_index.h"

namespace {

using Clock = std::chrono::steady_clock;

inline int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch())
      .count();
}

constexpr int kSlots = 3;           // batches in flight (GPU running / collected / collecting)
constexpr int kMaxTerms = 256;      // sparse terms per query (armi_sparse_topk's limit)
// Result ring entries (tickets whose results stay readable): the largest power of two whose
// payload fits 128 MiB of host memory (2^19 tickets at k = 10), at least 2^14 and 64 * max_batch.
// A caller that lets a ticket fall a whole ring behind gets "result overwritten" from
// armi_stream_wait, never another ticket's results (the entries are published seqlock-style).
int64_t ring_entries(int max_batch, int k) {
  const int64_t per = (int64_t)k * (4 + 8 + 8) + (int64_t)sizeof(int64_t) * 6;
  int64_t r = 1 << 14;
  while (r * 2 * per <= (int64_t(128) << 20)) r <<= 1;
  while (r < 64 * (int64_t)max_batch) r <<= 1;
  return r;
}

struct Slot {
  int n = 0;                         // queries in the batch
  int64_t first_ticket = 0;
  uint16_t* h_queries = nullptr;     // pinned [max_batch][dim]
  uint16_t* d_queries = nullptr;
  float* d_scores = nullptr;
  int64_t* d_ids = nullptr;
  double* d_rank = nullptr;
  int32_t* d_count = nullptr;
  uint32_t* d_flags = nullptr;
  void* d_ws = nullptr;
  float* h_scores = nullptr;         // pinned results
  int64_t* h_ids = nullptr;
  double* h_rank = nullptr;
  int32_t* h_count = nullptr;
  hipEvent_t done = nullptr;
  int status = ARMI_OK;
  std::vector<int64_t> t_submit;     // [max_batch] submit time of each query
  std::vector<int32_t> qmode;        // [max_batch] branch (0 dense, 1 hybrid, 2 sparse)
  const uint64_t* mask = nullptr;    // the batch's row filter (every query of the batch)
  bool sealed = false;               // closed early: the next query needs another mask
  // hybrid servers: the batch's sparse query CSR (pinned + device), prefetch lists, fusion
  int nnz = 0;
  int32_t* h_sp_ptr = nullptr;       // [max_batch + 1]
  int32_t* h_sp_idx = nullptr;       // [max_batch * kMaxTerms]
  float* h_sp_val = nullptr;
  int32_t* d_sp_ptr = nullptr;
  int32_t* d_sp_idx = nullptr;
  float* d_sp_val = nullptr;
  float* d_sp_scores = nullptr;      // [max_batch][2k]
  int64_t* d_sp_ids = nullptr;
  int32_t* d_sp_count = nullptr;
  uint32_t* d_sp_flags = nullptr;
  float* h_sp_scores = nullptr;      // pinned sparse lists (sparse-only queries)
  int64_t* h_sp_ids = nullptr;
  int32_t* h_sp_count = nullptr;
  void* d_sp_ws = nullptr;
  int64_t* d_f_ids = nullptr;        // fused [max_batch][k]
  double* d_f_score = nullptr;
  int32_t* d_f_count = nullptr;
  int64_t* h_f_ids = nullptr;
  double* h_f_score = nullptr;
  int32_t* h_f_count = nullptr;
};

// A ring entry is published seqlock-style: the completion thread sets ticket to kWriting, writes
// the payload (fields + the r_* arrays), then stores the ticket with release; a reader copies the
// payload after an acquire load equal to its ticket and re-checks the ticket afterwards.
constexpr int64_t kWriting = -2;

struct Entry {
  std::atomic<int64_t> ticket{-1};   // ticket whose result this entry holds (complete when set)
  int64_t t_submit = 0;
  int64_t t_done = 0;
  int32_t count = 0;
  int32_t mode = 0;                  // 0 dense branch, 1 hybrid (RRF scores in rank), 2 sparse
  int status = ARMI_OK;
};

}  // namespace

struct armi_stream {
  const armi_index* idx = nullptr;
  const armi_sparse_index* sidx = nullptr;  // non-null: hybrid server
  int rrf_k = 2;
  int kp = 0;                               // dense prefetch limit (2k hybrid, k dense)
  size_t sws_bytes = 0;
  int k = 0, max_batch = 0, dim = 0;
  int64_t max_wait_ns = 0;
  size_t ws_bytes = 0;
  hipStream_t stream = nullptr;
  Slot slots[kSlots];
  // result ring: entries + their payload arrays
  std::vector<Entry> ring;
  std::vector<float> r_scores;
  std::vector<int64_t> r_ids;
  std::vector<double> r_rank;
  // collection state (mu)
  std::mutex mu;
  std::condition_variable cv_dispatch;   // dispatcher: batch ready / stop
  std::condition_variable cv_space;      // submitters: a collecting slot is free
  std::condition_variable cv_complete;   // completion thread: a launched slot to finish
  std::condition_variable cv_done;       // waiters: results published
  int collect = 0;                       // slot being filled
  int64_t first_submit_ns = 0;           // submit time of its first query
  std::deque<int> launched;              // slots on the GPU, in order
  int free_slots = kSlots - 1;           // slots neither collecting nor launched
  int64_t next_ticket = 0;
  bool stop = false;
  std::atomic<int64_t> batches{0}, queries{0};
  std::thread dispatcher, completer;
  int device = 0;
  int64_t ring_n = 0;                    // ring entries (a power of two)
  std::atomic<int> active{0};            // callers inside submit / wait / stats / loadgen
};

namespace {

int launch_slot(armi_stream* s, Slot& sl) {
  const size_t qbytes = (size_t)sl.n * s->dim * sizeof(uint16_t);
  ARMI_HIP(hipMemcpyAsync(sl.d_queries, sl.h_queries, qbytes, hipMemcpyHostToDevice, s->stream));
  int rc = armi_dense_topk(s->idx, sl.d_queries, sl.n, s->kp, sl.mask, sl.d_scores, sl.d_ids,
                           sl.d_rank, sl.d_count, sl.d_flags, sl.d_ws, s->ws_bytes, s->stream);
  if (rc != ARMI_OK) return rc;
  if (s->sidx && sl.nnz > 0) {  // (no query of the batch has terms: every answer is dense)
    ARMI_HIP(hipMemcpyAsync(sl.d_sp_ptr, sl.h_sp_ptr, (size_t)(sl.n + 1) * sizeof(int32_t),
                            hipMemcpyHostToDevice, s->stream));
    if (sl.nnz > 0) {
      ARMI_HIP(hipMemcpyAsync(sl.d_sp_idx, sl.h_sp_idx, (size_t)sl.nnz * sizeof(int32_t),
                              hipMemcpyHostToDevice, s->stream));
      ARMI_HIP(hipMemcpyAsync(sl.d_sp_val, sl.h_sp_val, (size_t)sl.nnz * sizeof(float),
                              hipMemcpyHostToDevice, s->stream));
    }
    rc = armi_sparse_topk(s->sidx, sl.d_sp_ptr, sl.d_sp_idx, sl.d_sp_val, sl.n, s->kp, sl.mask,
                          sl.d_sp_scores, sl.d_sp_ids, sl.d_sp_count, sl.d_sp_flags, sl.d_sp_ws,
                          s->sws_bytes, s->stream);
    if (rc != ARMI_OK) return rc;
    rc = armi_rrf_fuse(sl.d_ids, sl.d_count, s->kp, sl.d_sp_ids, sl.d_sp_count, s->kp, sl.n,
                       s->rrf_k, s->k, sl.d_f_ids, sl.d_f_score, sl.d_f_count, s->stream);
    if (rc != ARMI_OK) return rc;
    const size_t nf = (size_t)sl.n * s->k;
    ARMI_HIP(hipMemcpyAsync(sl.h_f_ids, sl.d_f_ids, nf * sizeof(int64_t), hipMemcpyDeviceToHost,
                            s->stream));
    ARMI_HIP(hipMemcpyAsync(sl.h_f_score, sl.d_f_score, nf * sizeof(double),
                            hipMemcpyDeviceToHost, s->stream));
    ARMI_HIP(hipMemcpyAsync(sl.h_f_count, sl.d_f_count, (size_t)sl.n * sizeof(int32_t),
                            hipMemcpyDeviceToHost, s->stream));
    const size_t ns = (size_t)sl.n * s->kp;
    ARMI_HIP(hipMemcpyAsync(sl.h_sp_scores, sl.d_sp_scores, ns * sizeof(float),
                            hipMemcpyDeviceToHost, s->stream));
    ARMI_HIP(hipMemcpyAsync(sl.h_sp_ids, sl.d_sp_ids, ns * sizeof(int64_t), hipMemcpyDeviceToHost,
                            s->stream));
    ARMI_HIP(hipMemcpyAsync(sl.h_sp_count, sl.d_sp_count, (size_t)sl.n * sizeof(int32_t),
                            hipMemcpyDeviceToHost, s->stream));
  }
  const size_t nk = (size_t)sl.n * s->kp;
  ARMI_HIP(hipMemcpyAsync(sl.h_scores, sl.d_scores, nk * sizeof(float), hipMemcpyDeviceToHost,
                          s->stream));
  ARMI_HIP(hipMemcpyAsync(sl.h_ids, sl.d_ids, nk * sizeof(int64_t), hipMemcpyDeviceToHost,
                          s->stream));
  ARMI_HIP(hipMemcpyAsync(sl.h_rank, sl.d_rank, nk * sizeof(double), hipMemcpyDeviceToHost,
                          s->stream));
  ARMI_HIP(hipMemcpyAsync(sl.h_count, sl.d_count, (size_t)sl.n * sizeof(int32_t),
                          hipMemcpyDeviceToHost, s->stream));
  ARMI_HIP(hipEventRecord(sl.done, s->stream));
  return ARMI_OK;
}

void dispatcher_main(armi_stream* s) {
  (void)hipSetDevice(s->device);
  std::unique_lock<std::mutex> lk(s->mu);
  for (;;) {
    // a batch is due when full, or when its first query has waited max_wait
    for (;;) {
      if (s->stop) return;
      Slot& c = s->slots[s->collect];
      if (c.n == s->max_batch || c.sealed) break;
      if (c.n > 0) {
        const int64_t due = s->first_submit_ns + s->max_wait_ns;
        const int64_t t = now_ns();
        if (t >= due) break;
        s->cv_dispatch.wait_for(lk, std::chrono::nanoseconds(due - t));
      } else {
        s->cv_dispatch.wait(lk);
      }
    }
    // hand the batch over, and open the next collecting slot (wait for one if all are busy)
    while (s->free_slots == 0 && !s->stop) s->cv_dispatch.wait(lk);
    if (s->stop) return;
    const int cur = s->collect;
    int nxt = (cur + 1) % kSlots;
    s->collect = nxt;
    --s->free_slots;
    Slot& sl = s->slots[cur];
    lk.unlock();
    s->cv_space.notify_all();
    sl.status = launch_slot(s, sl);
    lk.lock();
    s->launched.push_back(cur);
    s->cv_complete.notify_one();
  }
}

void completer_main(armi_stream* s) {
  (void)hipSetDevice(s->device);
  std::unique_lock<std::mutex> lk(s->mu);
  for (;;) {
    while (s->launched.empty() && !s->stop) s->cv_complete.wait(lk);
    if (s->launched.empty() && s->stop) return;
    const int cur = s->launched.front();
    lk.unlock();
    Slot& sl = s->slots[cur];
    int status = sl.status;
    if (status == ARMI_OK && hipEventSynchronize(sl.done) != hipSuccess) status = ARMI_ERR_HIP;
    const int64_t t = now_ns();
    for (int i = 0; i < sl.n; ++i) {
      const int64_t tk = sl.first_ticket + i;
      Entry& e = s->ring[tk % s->ring_n];
      const size_t o = (size_t)(tk % s->ring_n) * s->k;
      const int qm = sl.qmode[i];
      e.ticket.store(kWriting, std::memory_order_relaxed);
      std::atomic_thread_fence(std::memory_order_release);
      // (sl.nnz == 0: the batch's sparse pass did not run; its hybrid / sparse-only queries
      // carry empty sparse vectors: RRF over the dense list alone / an empty result, exactly
      // what the device pass gives an empty query)
      if (status == ARMI_OK && qm != 0 && sl.nnz == 0) {
        const size_t d = (size_t)i * s->kp;
        e.count = qm == 1 ? std::min(sl.h_count[i], s->k) : 0;
        for (int j = 0; j < s->k; ++j) {
          const bool v = j < e.count;
          const double rrf = 1.0 / (double)(s->rrf_k + j);
          s->r_ids[o + j] = v ? sl.h_ids[d + j] : -1;
          s->r_rank[o + j] = v ? rrf : 0.0;
          s->r_scores[o + j] = v ? (float)rrf : 0.0f;
        }
        e.mode = qm;
      } else if (status == ARMI_OK && qm == 2) {
        // sparse-only branch: the first k of the sparse prefetch list, hit.score = the dot
        const size_t d = (size_t)i * s->kp;
        e.count = std::min(sl.h_sp_count[i], s->k);
        for (int j = 0; j < s->k; ++j) {
          s->r_ids[o + j] = sl.h_sp_ids[d + j];
          s->r_scores[o + j] = sl.h_sp_scores[d + j];
          s->r_rank[o + j] = (double)sl.h_sp_scores[d + j];
        }
        e.mode = 2;
      } else if (status == ARMI_OK && qm == 1) {
        // hybrid branch: the fused list, hit.score = the RRF score (rank holds it in fp64)
        const size_t f = (size_t)i * s->k;
        e.count = sl.h_f_count[i];
        for (int j = 0; j < s->k; ++j) {
          s->r_ids[o + j] = sl.h_f_ids[f + j];
          s->r_rank[o + j] = sl.h_f_score[f + j];
          s->r_scores[o + j] = (float)sl.h_f_score[f + j];
        }
        e.mode = 1;
      } else if (status == ARMI_OK) {
        // dense branch: the first k of the dense list (prefetch 2k on a hybrid server)
        const size_t d = (size_t)i * s->kp;
        std::memcpy(&s->r_scores[o], sl.h_scores + d, s->k * sizeof(float));
        std::memcpy(&s->r_ids[o], sl.h_ids + d, s->k * sizeof(int64_t));
        std::memcpy(&s->r_rank[o], sl.h_rank + d, s->k * sizeof(double));
        e.count = std::min(sl.h_count[i], s->k);
        e.mode = 0;
      } else {
        e.count = 0;
      }
      e.status = status;
      e.t_submit = sl.t_submit[i];
      e.t_done = t;
      e.ticket.store(tk, std::memory_order_release);
    }
    s->batches.fetch_add(1);
    s->queries.fetch_add(sl.n);
    lk.lock();
    sl.n = 0;
    sl.nnz = 0;
    sl.mask = nullptr;
    sl.sealed = false;
    s->launched.pop_front();
    ++s->free_slots;
    s->cv_done.notify_all();
    s->cv_dispatch.notify_one();
  }
}

void free_slot(Slot& sl) {
  if (sl.h_queries) (void)hipHostFree(sl.h_queries);
  if (sl.h_scores) (void)hipHostFree(sl.h_scores);
  if (sl.h_ids) (void)hipHostFree(sl.h_ids);
  if (sl.h_rank) (void)hipHostFree(sl.h_rank);
  if (sl.h_count) (void)hipHostFree(sl.h_count);
  for (void* p : {(void*)sl.h_sp_ptr, (void*)sl.h_sp_idx, (void*)sl.h_sp_val, (void*)sl.h_f_ids,
                  (void*)sl.h_f_score, (void*)sl.h_f_count, (void*)sl.h_sp_scores,
                  (void*)sl.h_sp_ids, (void*)sl.h_sp_count})
    if (p) (void)hipHostFree(p);
  for (void* p : {(void*)sl.d_queries, (void*)sl.d_scores, (void*)sl.d_ids, (void*)sl.d_rank,
                  (void*)sl.d_count, (void*)sl.d_flags, sl.d_ws, (void*)sl.d_sp_ptr,
                  (void*)sl.d_sp_idx, (void*)sl.d_sp_val, (void*)sl.d_sp_scores,
                  (void*)sl.d_sp_ids, (void*)sl.d_sp_count, (void*)sl.d_sp_flags, sl.d_sp_ws,
                  (void*)sl.d_f_ids, (void*)sl.d_f_score, (void*)sl.d_f_count})
    if (p) (void)hipFree(p);
  if (sl.done) (void)hipEventDestroy(sl.done);
  sl = Slot{};
}

void shutdown(armi_stream* s) {
  {
    std::lock_guard<std::mutex> g(s->mu);
    s->stop = true;
  }
  s->cv_dispatch.notify_all();
  s->cv_complete.notify_all();
  s->cv_space.notify_all();
  if (s->dispatcher.joinable()) s->dispatcher.join();
  if (s->completer.joinable()) s->completer.join();
  {
    std::lock_guard<std::mutex> g(s->mu);
    s->cv_done.notify_all();
  }
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  for (auto& sl : s->slots) free_slot(sl);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  s->stream = nullptr;
}

int alloc_slot(armi_stream* s, Slot& sl) {
  const size_t nq = (size_t)s->max_batch, nk = nq * s->kp;
  ARMI_HIP(hipHostMalloc(reinterpret_cast<void**>(&sl.h_queries), nq * s->dim * 2));
  ARMI_HIP(hipHostMalloc(reinterpret_cast<void**>(&sl.h_scores), nk * sizeof(float)));
  ARMI_HIP(hipHostMalloc(reinterpret_cast<void**>(&sl.h_ids), nk * sizeof(int64_t)));
  ARMI_HIP(hipHostMalloc(reinterpret_cast<void**>(&sl.h_rank), nk * sizeof(double)));
  ARMI_HIP(hipHostMalloc(reinterpret_cast<void**>(&sl.h_count), nq * sizeof(int32_t)));
  ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&sl.d_queries), nq * s->dim * 2));
  ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&sl.d_scores), nk * sizeof(float)));
  ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&sl.d_ids), nk * sizeof(int64_t)));
  ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&sl.d_rank), nk * sizeof(double)));
  ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&sl.d_count), nq * sizeof(int32_t)));
  ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&sl.d_flags), nq * sizeof(uint32_t)));
  ARMI_HIP(hipMalloc(&sl.d_ws, s->ws_bytes));
  ARMI_HIP(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
  sl.t_submit.assign(nq, 0);
  sl.qmode.assign(nq, 0);
  if (s->sidx) {
    const size_t nt = nq * kMaxTerms, nf = nq * s->k;
    ARMI_HIP(hipHostMalloc(reinterpret_cast<void**>(&sl.h_sp_ptr), (nq + 1) * sizeof(int32_t)));
    ARMI_HIP(hipHostMalloc(reinterpret_cast<void**>(&sl.h_sp_idx), nt * sizeof(int32_t)));
    ARMI_HIP(hipHostMalloc(reinterpret_cast<void**>(&sl.h_sp_val), nt * sizeof(float)));
    ARMI_HIP(hipHostMalloc(reinterpret_cast<void**>(&sl.h_f_ids), nf * sizeof(int64_t)));
    ARMI_HIP(hipHostMalloc(reinterpret_cast<void**>(&sl.h_f_score), nf * sizeof(double)));
    ARMI_HIP(hipHostMalloc(reinterpret_cast<void**>(&sl.h_f_count), nq * sizeof(int32_t)));
    ARMI_HIP(hipHostMalloc(reinterpret_cast<void**>(&sl.h_sp_scores), nk * sizeof(float)));
    ARMI_HIP(hipHostMalloc(reinterpret_cast<void**>(&sl.h_sp_ids), nk * sizeof(int64_t)));
    ARMI_HIP(hipHostMalloc(reinterpret_cast<void**>(&sl.h_sp_count), nq * sizeof(int32_t)));
    ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&sl.d_sp_ptr), (nq + 1) * sizeof(int32_t)));
    ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&sl.d_sp_idx), nt * sizeof(int32_t)));
    ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&sl.d_sp_val), nt * sizeof(float)));
    ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&sl.d_sp_scores), nk * sizeof(float)));
    ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&sl.d_sp_ids), nk * sizeof(int64_t)));
    ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&sl.d_sp_count), nq * sizeof(int32_t)));
    ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&sl.d_sp_flags), nq * sizeof(uint32_t)));
    ARMI_HIP(hipMalloc(&sl.d_sp_ws, s->sws_bytes));
    ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&sl.d_f_ids), nf * sizeof(int64_t)));
    ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&sl.d_f_score), nf * sizeof(double)));
    ARMI_HIP(hipMalloc(reinterpret_cast<void**>(&sl.d_f_count), nq * sizeof(int32_t)));
    sl.h_sp_ptr[0] = 0;
  }
  return ARMI_OK;
}

}  // namespace

namespace {

int create_impl(const armi_index* idx, const armi_sparse_index* sidx, int k, int rrf_k,
                int max_batch, double max_wait_us, armi_stream** out) {
  ARMI_REQUIRE(idx && out, "armi_stream_create: null pointer argument");
  ARMI_REQUIRE(k >= 1 && k <= (sidx ? 120 : 240), "armi_stream_create: k out of range");
  ARMI_REQUIRE(max_batch >= 1 && max_batch <= 4096, "armi_stream_create: max_batch in [1, 4096]");
  ARMI_REQUIRE(max_wait_us >= 0.0, "armi_stream_create: max_wait_us < 0");
  ARMI_REQUIRE(rrf_k >= 1, "armi_stream_create: rrf_k must be >= 1");
  *out = nullptr;
  auto* s = new armi_stream();
  s->idx = idx;
  s->sidx = sidx;
  s->rrf_k = rrf_k;
  s->k = k;
  s->kp = sidx ? 2 * k : k;
  s->max_batch = max_batch;
  s->dim = armi_index_dim(idx);
  s->max_wait_ns = (int64_t)(max_wait_us * 1e3);
  s->device = idx->device;
  s->ws_bytes = armi_dense_workspace_bytes(idx, max_batch, s->kp);
  if (sidx) s->sws_bytes = armi_sparse_workspace_bytes(sidx, max_batch, s->kp);
  s->ring_n = ring_entries(max_batch, k);
  s->ring = std::vector<Entry>(s->ring_n);
  s->r_scores.assign((size_t)s->ring_n * k, 0.f);
  s->r_ids.assign((size_t)s->ring_n * k, -1);
  s->r_rank.assign((size_t)s->ring_n * k, 0.0);
  int rc = ARMI_OK;
  if (hipSetDevice(s->device) != hipSuccess ||
      hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
    rc = armi::fail(ARMI_ERR_HIP, "armi_stream_create: stream");
  }
  for (int i = 0; i < kSlots && rc == ARMI_OK; ++i) rc = alloc_slot(s, s->slots[i]);
  if (rc != ARMI_OK) {
    shutdown(s);
    delete s;
    return rc;
  }
  s->dispatcher = std::thread(dispatcher_main, s);
  s->completer = std::thread(completer_main, s);
  *out = s;
  return ARMI_OK;
}

// Counts a caller inside the server's entry points; armi_stream_destroy waits for the count to
// drop to zero before it frees anything.
struct Active {
  armi_stream* s;
  explicit Active(armi_stream* s_) : s(s_) { if (s) s->active.fetch_add(1); }
  ~Active() { if (s) s->active.fetch_sub(1); }
};

// Stops the server: no new batches, every waiter and blocked submitter wakes and returns.
void stop_impl(armi_stream* s) {
  {
    std::lock_guard<std::mutex> g(s->mu);
    s->stop = true;
  }
  s->cv_dispatch.notify_all();
  s->cv_complete.notify_all();
  s->cv_space.notify_all();
  s->cv_done.notify_all();
}

int submit_impl(armi_stream* s, const uint16_t* query, const int32_t* sp_idx,
                const float* sp_val, int nnz, int mode, const uint64_t* mask, int64_t* ticket) {
  ARMI_REQUIRE(s && query && ticket, "armi_stream_submit: null pointer argument");
  ARMI_REQUIRE(nnz >= 0 && nnz <= kMaxTerms, "armi_stream_submit: nnz must be in [0, 256]");
  ARMI_REQUIRE(nnz == 0 || (s->sidx && sp_idx && sp_val),
               "armi_stream_submit: sparse terms need a hybrid server and both arrays");
  ARMI_REQUIRE(mode == ARMI_STREAM_AUTO || mode == ARMI_STREAM_DENSE || mode == ARMI_STREAM_SPARSE,
               "armi_stream_submit: unknown mode");
  // the branch (QdrantRetriever.search, qdrant.py:272/299): a query that carries a sparse vector
  // (the arrays are non-null, even with nnz = 0: `if query.sparse` is true for an empty
  // SparseVector object) takes the hybrid / sparse-only branch, else the dense one
  const bool has_sparse = sp_idx != nullptr && sp_val != nullptr;
  const int qm = !has_sparse || !s->sidx || mode == ARMI_STREAM_DENSE
                     ? 0 : (mode == ARMI_STREAM_SPARSE ? 2 : 1);
  if (qm == 0) nnz = 0;  // a dense-branch query adds nothing to the batch's sparse pass
  std::unique_lock<std::mutex> lk(s->mu);
  for (;;) {
    if (s->stop) return armi::fail(ARMI_ERR_INVALID, "armi_stream_submit: server stopped");
    Slot& c = s->slots[s->collect];
    if (c.n > 0 && !c.sealed && c.mask != mask) {  // another filter: close the collecting batch
      c.sealed = true;
      s->cv_dispatch.notify_one();
    }
    if (!c.sealed && c.n < s->max_batch) break;
    s->cv_space.wait(lk);  // collecting batch full (or sealed) and not yet handed over
  }
  Slot& c = s->slots[s->collect];
  const int64_t tk = s->next_ticket++;
  if (c.n == 0) {
    c.first_ticket = tk;
    c.mask = mask;
    s->first_submit_ns = now_ns();
  }
  std::memcpy(c.h_queries + (size_t)c.n * s->dim, query, (size_t)s->dim * sizeof(uint16_t));
  if (s->sidx) {
    if (nnz > 0) {
      std::memcpy(c.h_sp_idx + c.nnz, sp_idx, (size_t)nnz * sizeof(int32_t));
      std::memcpy(c.h_sp_val + c.nnz, sp_val, (size_t)nnz * sizeof(float));
    }
    c.nnz += nnz;
    c.h_sp_ptr[c.n + 1] = c.nnz;
  }
  c.qmode[c.n] = qm;
  c.t_submit[c.n] = now_ns();
  ++c.n;
  const bool wake = c.n == 1 || c.n == s->max_batch;
  lk.unlock();
  if (wake) s->cv_dispatch.notify_one();
  *ticket = tk;
  return ARMI_OK;
}

// Waits for `ticket` and copies its result out; t_submit / t_done (nullable) receive its submit
// and completion times. The copy is validated after the fact: if the completion thread reused
// the entry meanwhile (the caller fell a whole ring behind), the call fails instead of returning
// another ticket's results.
int wait_impl(armi_stream* s, int64_t ticket, float* scores, int64_t* ids, double* rank,
              int32_t* count, int32_t* mode, double timeout_us, int64_t* t_submit,
              int64_t* t_done) {
  ARMI_REQUIRE(s && count, "armi_stream_wait: null pointer argument");
  ARMI_REQUIRE(ticket >= 0, "armi_stream_wait: bad ticket");
  Entry& e = s->ring[ticket % s->ring_n];
  if (e.ticket.load(std::memory_order_acquire) != ticket) {
    std::unique_lock<std::mutex> lk(s->mu);
    const auto until = Clock::now() + std::chrono::nanoseconds((int64_t)(timeout_us * 1e3));
    while (e.ticket.load(std::memory_order_acquire) != ticket) {
      if (ticket >= s->next_ticket) return armi::fail(ARMI_ERR_INVALID, "armi_stream_wait: unknown ticket");
      if (e.ticket.load(std::memory_order_acquire) > ticket)
        return armi::fail(ARMI_ERR_INVALID, "armi_stream_wait: result overwritten (ring wrapped)");
      if (s->stop) return armi::fail(ARMI_ERR_INVALID, "armi_stream_wait: server stopped");
      if (s->cv_done.wait_until(lk, until) == std::cv_status::timeout &&
          e.ticket.load(std::memory_order_acquire) != ticket)
        return armi::fail(ARMI_ERR_INVALID, "armi_stream_wait: timeout");
    }
  }
  const int status = e.status;
  const int32_t cnt = e.count, md = e.mode;
  const int64_t ts = e.t_submit, td = e.t_done;
  const size_t o = (size_t)(ticket % s->ring_n) * s->k;
  if (status == ARMI_OK) {
    if (scores) std::memcpy(scores, &s->r_scores[o], s->k * sizeof(float));
    if (ids) std::memcpy(ids, &s->r_ids[o], s->k * sizeof(int64_t));
    if (rank) std::memcpy(rank, &s->r_rank[o], s->k * sizeof(double));
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  if (e.ticket.load(std::memory_order_relaxed) != ticket)
    return armi::fail(ARMI_ERR_INVALID, "armi_stream_wait: result overwritten (ring wrapped)");
  if (status != ARMI_OK) return armi::fail(status, "armi_stream_wait: the batch failed");
  if (mode) *mode = md;
  *count = cnt;
  if (t_submit) *t_submit = ts;
  if (t_done) *t_done = td;
  return ARMI_OK;
}

}  // namespace

extern "C" {

int armi_stream_create(const armi_index* idx, int k, int max_batch, double max_wait_us,
                       armi_stream** out) {
  return create_impl(idx, nullptr, k, 2, max_batch, max_wait_us, out);
}

int armi_stream_create_hybrid(const armi_index* idx, const armi_sparse_index* sidx, int k,
                              int rrf_k, int max_batch, double max_wait_us, armi_stream** out) {
  ARMI_REQUIRE(sidx, "armi_stream_create_hybrid: sparse index is null");
  return create_impl(idx, sidx, k, rrf_k, max_batch, max_wait_us, out);
}

int armi_stream_stop(armi_stream* s) {
  ARMI_REQUIRE(s, "armi_stream_stop: null server");
  stop_impl(s);
  return ARMI_OK;
}

int armi_stream_destroy(armi_stream* s) {
  if (!s) return ARMI_OK;
  stop_impl(s);
  // callers still inside wait / submit (woken by the stop) leave before anything is freed
  while (s->active.load() > 0) {
    {
      std::lock_guard<std::mutex> g(s->mu);
      s->cv_done.notify_all();
      s->cv_space.notify_all();
    }
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  shutdown(s);
  delete s;
  return ARMI_OK;
}

int armi_stream_submit(armi_stream* s, const uint16_t* query, int64_t* ticket) {
  Active a(s);
  return submit_impl(s, query, nullptr, nullptr, 0, ARMI_STREAM_AUTO, nullptr, ticket);
}

int armi_stream_submit_hybrid(armi_stream* s, const uint16_t* query, const int32_t* sp_indices,
                              const float* sp_values, int nnz, int64_t* ticket) {
  Active a(s);
  return submit_impl(s, query, sp_indices, sp_values, nnz, ARMI_STREAM_AUTO, nullptr, ticket);
}

int armi_stream_submit_ex(armi_stream* s, const uint16_t* query, const int32_t* sp_indices,
                          const float* sp_values, int nnz, int mode, const uint64_t* row_mask,
                          int64_t* ticket) {
  Active a(s);
  return submit_impl(s, query, sp_indices, sp_values, nnz, mode, row_mask, ticket);
}

int armi_stream_wait(armi_stream* s, int64_t ticket, float* scores, int64_t* ids, double* rank,
                     int32_t* count, int32_t* mode, double timeout_us) {
  Active a(s);
  return wait_impl(s, ticket, scores, ids, rank, count, mode, timeout_us, nullptr, nullptr);
}

int armi_stream_stats(armi_stream* s, int64_t* batches, int64_t* queries) {
  ARMI_REQUIRE(s && batches && queries, "armi_stream_stats: null pointer argument");
  Active a(s);
  *batches = s->batches.load();
  *queries = s->queries.load();
  return ARMI_OK;
}

int armi_stream_loadgen(armi_stream* s, const uint16_t* queries, const int32_t* q_indptr,
                        const int32_t* q_indices, const float* q_values, int64_t n_vectors,
                        int64_t n_queries, double qps, uint64_t seed, double* latency_us,
                        double* elapsed_s, int64_t* completed, int64_t* out_ids,
                        int32_t* out_count) {
  ARMI_REQUIRE(s && queries && latency_us && elapsed_s && completed,
               "armi_stream_loadgen: null pointer argument");
  ARMI_REQUIRE(n_vectors >= 1, "armi_stream_loadgen: n_vectors < 1");
  ARMI_REQUIRE(n_queries >= 1, "armi_stream_loadgen: n_queries < 1");
  ARMI_REQUIRE(qps > 0.0, "armi_stream_loadgen: qps must be > 0");
  Active a(s);
  std::mt19937_64 rng(seed);
  std::exponential_distribution<double> gap(qps);
  std::vector<int64_t> tickets((size_t)n_queries);
  std::atomic<int64_t> n_sub{0};
  // results are collected in ticket order while arrivals continue, so only the tickets in flight
  // (<= kSlots batches plus the collector's lag) need to stay in the result ring
  int64_t t_last = 0, t_first = -1;
  std::atomic<int> rc_col{ARMI_OK};
  std::thread collector([&] {
    int32_t cnt = 0;
    for (int64_t i = 0; i < n_queries; ++i) {
      while (n_sub.load(std::memory_order_acquire) <= i) {
        if (rc_col.load() != ARMI_OK) return;
        std::this_thread::sleep_for(std::chrono::microseconds(5));
      }
      const int64_t tk = tickets[(size_t)i];
      int64_t* ids = out_ids ? out_ids + (size_t)i * s->k : nullptr;
      int64_t ts = 0, td = 0;
      if (int rc = wait_impl(s, tk, nullptr, ids, nullptr, &cnt, nullptr, 60e6, &ts, &td)) {
        rc_col.store(rc);
        return;
      }
      if (out_count) out_count[i] = cnt;
      latency_us[i] = (double)(td - ts) * 1e-3;
      t_last = std::max(t_last, td);
      if (t_first < 0) t_first = ts;
    }
  });
  const int64_t t0 = now_ns();
  double due = 0.0;  // seconds since t0
  int rc = ARMI_OK;
  for (int64_t i = 0; i < n_queries && rc == ARMI_OK && rc_col.load() == ARMI_OK; ++i) {
    due += gap(rng);
    const int64_t due_ns = t0 + (int64_t)(due * 1e9);
    for (;;) {  // open-loop arrivals: sleep to ~50 us before the due time, then spin
      const int64_t t = now_ns();
      if (t >= due_ns) break;
      if (due_ns - t > 100000) std::this_thread::sleep_for(std::chrono::nanoseconds(due_ns - t - 50000));
    }
    const int64_t v = i % n_vectors;
    const int nnz = q_indptr ? q_indptr[v + 1] - q_indptr[v] : 0;
    rc = submit_impl(s, queries + (size_t)v * s->dim, q_indptr ? q_indices + q_indptr[v] : nullptr,
                     q_indptr ? q_values + q_indptr[v] : nullptr, nnz, ARMI_STREAM_AUTO, nullptr,
                     &tickets[(size_t)i]);
    if (rc == ARMI_OK) n_sub.store(i + 1, std::memory_order_release);
  }
  if (rc != ARMI_OK) rc_col.store(rc);  // stops the collector
  collector.join();
  if (rc != ARMI_OK) return rc;
  if (rc_col.load() != ARMI_OK)
    return armi::fail(rc_col.load(), "armi_stream_loadgen: waiting for a result failed");
  *elapsed_s = (double)(t_last - t_first) * 1e-9;
  *completed = n_queries;
  return ARMI_OK;
}

}  // extern "C"
