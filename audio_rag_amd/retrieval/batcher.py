"""Streaming query front end: concurrent callers' searches coalesced into device batches.

The reference answers one query per request: the REST layer calls pipeline.query() once per
request in each of its 4 uvicorn processes (src/audio_rag/api/v1/query.py:90-115,
Dockerfile.api:85-86), so Qdrant sees batch-1 searches. On the MI355X a batch-1 scan costs the
same HBM pass as a batch-64 scan, so a server must batch across requests. QueryBatcher is that
layer (BASELINE config 5 "streaming query at fixed QPS"): callers
submit single queries from any thread and get a Future of the reference-shaped
list[RetrievalResult]; one worker thread drains the queue into batches of up to max_batch
queries, waiting at most max_wait_ms after the first arrival, and runs one
MI355XRetriever.search_batch per (filter, has-sparse) group. Per-query semantics are those of
MI355XRetriever.search (qdrant.py:227-352); only the grouping is new.
"""

from __future__ import annotations

import logging
import queue
import threading
import time
import weakref
from concurrent.futures import Future
from dataclasses import dataclass, field

import numpy as np
import torch

from audio_rag_amd.core.base import EmbeddingResult, RetrievalResult
from audio_rag_amd.core.exceptions import RetrievalError
from audio_rag_amd.retrieval.mi355x import MI355XRetriever, QueryBatch, query_sparse_arrays

logger = logging.getLogger(__name__)


@dataclass
class _Request:
    dense: np.ndarray                       # float16 [dim]
    sparse: tuple[np.ndarray, np.ndarray] | None
    filter_metadata: dict | None
    future: Future
    t_submit: float = field(default_factory=time.perf_counter)


def _filter_key(f: dict | None):
    return None if not f else tuple(sorted((k, repr(v)) for k, v in f.items()))


def _sorted_terms(indices, values) -> tuple[np.ndarray, np.ndarray]:
    """A query's sparse terms as the device search needs them: ascending unique int32 indices
    (Qdrant stores sparse vectors sorted by index and rejects duplicates)."""
    idx = np.asarray(indices, dtype=np.int64).reshape(-1)
    val = np.asarray(values, dtype=np.float32).reshape(-1)
    if idx.shape != val.shape:
        raise RetrievalError("sparse query indices and values differ in length")
    order = np.argsort(idx, kind="stable")
    idx, val = idx[order], val[order]
    if idx.size and (np.any(idx[1:] == idx[:-1]) or idx[0] < 0 or idx[-1] >= 2**31):
        raise RetrievalError("sparse query indices must be unique non-negative int32")
    return np.ascontiguousarray(idx, dtype=np.int32), np.ascontiguousarray(val)


def _sorted_csr(indptr, indices, values) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """_sorted_terms for every row of a query CSR at once."""
    indptr = np.asarray(indptr, dtype=np.int64)
    idx = np.asarray(indices, dtype=np.int64)
    val = np.asarray(values, dtype=np.float32)
    row = np.repeat(np.arange(indptr.size - 1), np.diff(indptr))
    order = np.lexsort((idx, row))
    idx, val = idx[order], val[order]
    if idx.size and (np.any((idx[1:] == idx[:-1]) & (row[1:] == row[:-1])) or idx.min() < 0
                     or idx.max() >= 2**31):
        raise RetrievalError("sparse query indices must be unique non-negative int32 per query")
    return (np.ascontiguousarray(indptr, dtype=np.int32), np.ascontiguousarray(idx, dtype=np.int32),
            np.ascontiguousarray(val))


class QueryBatcher:
    def __init__(self, retriever: MI355XRetriever, collection_name: str | None = None,
                 top_k: int | None = None, search_type: str | None = None, max_batch: int = 64,
                 max_wait_ms: float = 2.0):
        if max_batch < 1:
            raise ValueError("max_batch must be >= 1")
        self.retriever = retriever
        self.collection_name = collection_name
        self.top_k = top_k
        self.search_type = search_type
        self.max_batch = max_batch
        self.max_wait = max_wait_ms * 1e-3
        self._q: queue.Queue[_Request | None] = queue.Queue()
        self._closed = False
        self.batches = 0
        self.queries = 0
        self._worker = threading.Thread(target=self._run, name="armi-query-batcher", daemon=True)
        self._worker.start()

    # ------------------------------------------------------------------------ callers

    def submit_arrays(self, dense: np.ndarray, sparse: tuple[np.ndarray, np.ndarray] | None = None,
                      filter_metadata: dict | None = None) -> Future:
        """dense: [dim] query vector (cast to fp16 as the store holds it); sparse: (indices,
        values) or None. Returns a Future of list[RetrievalResult]."""
        if self._closed:
            raise RetrievalError("QueryBatcher is closed")
        fut: Future = Future()
        d = np.ascontiguousarray(dense, dtype=np.float16).reshape(-1)
        if sparse is not None:
            sparse = _sorted_terms(*sparse)
        self._q.put(_Request(d, sparse, filter_metadata, fut))
        return fut

    def submit(self, query: EmbeddingResult, filter_metadata: dict | None = None) -> Future:
        """EmbeddingResult (BGEM3Embedder.embed_query output) -> Future[list[RetrievalResult]]."""
        return self.submit_arrays(np.asarray(query.dense, dtype=np.float32),
                                  query_sparse_arrays(query.sparse), filter_metadata)

    def search(self, query: EmbeddingResult, filter_metadata: dict | None = None,
               timeout: float | None = None) -> list[RetrievalResult]:
        return self.submit(query, filter_metadata).result(timeout)

    def close(self) -> None:
        if not self._closed:
            self._closed = True
            self._q.put(None)
            self._worker.join()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ------------------------------------------------------------------------- worker

    def _collect(self, first: _Request) -> tuple[list[_Request], bool]:
        batch = [first]
        deadline = first.t_submit + self.max_wait
        stop = False
        while len(batch) < self.max_batch:
            wait = deadline - time.perf_counter()
            try:
                item = self._q.get(timeout=max(wait, 0.0)) if wait > 0 else self._q.get_nowait()
            except queue.Empty:
                break
            if item is None:
                stop = True
                break
            batch.append(item)
        return batch, stop

    def _run(self) -> None:
        if self.retriever.device.type == "cuda":
            torch.cuda.set_device(self.retriever.device)
        while True:
            first = self._q.get()
            if first is None:
                break
            batch, stop = self._collect(first)
            groups: dict = {}
            for r in batch:
                groups.setdefault((_filter_key(r.filter_metadata), r.sparse is not None), []).append(r)
            for reqs in groups.values():
                self._serve(reqs)
            if stop:
                break
        # fail whatever is left (closed while callers were still submitting)
        while True:
            try:
                item = self._q.get_nowait()
            except queue.Empty:
                break
            if item is not None and not item.future.done():
                item.future.set_exception(RetrievalError("QueryBatcher closed"))

    def _serve(self, reqs: list[_Request]) -> None:
        try:
            r = self.retriever
            dev = r.device
            dense = torch.from_numpy(np.stack([q.dense for q in reqs])).to(dev, non_blocking=True)
            qb = QueryBatch(dense=dense)
            if reqs[0].sparse is not None:
                indptr = np.zeros(len(reqs) + 1, dtype=np.int32)
                np.cumsum([len(q.sparse[0]) for q in reqs], out=indptr[1:])
                idx = np.concatenate([q.sparse[0] for q in reqs]).astype(np.int32)
                val = np.concatenate([q.sparse[1] for q in reqs]).astype(np.float32)
                t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
                qb = QueryBatch(dense=dense, sparse_indptr=t(indptr), sparse_indices=t(idx),
                                sparse_values=t(val))
            resolved = r._resolve_collection(self.collection_name)
            out, mode = r.search_batch(qb, self.top_k, resolved, reqs[0].filter_metadata,
                                       self.search_type)
            thr = None
            if mode == "legacy_dense" and r.config.score_threshold > 0:
                thr = r.config.score_threshold
            results = r.materialize_batch(out, mode, resolved, thr)
            for q, res in zip(reqs, results):
                q.future.set_result(res)
            self.batches += 1
            self.queries += len(reqs)
        except Exception as e:  # every caller of the batch sees the failure, as search() raises
            err = e if isinstance(e, RetrievalError) else RetrievalError(f"Search failed: {e}")
            for q in reqs:
                if not q.future.done():
                    q.future.set_exception(err)


class StreamServer:
    """The native streaming server (libarmi armi_stream_*, include/armi.h) over one collection's
    indexes: no Python thread in the request path. Callers submit single queries from any
    thread (ctypes releases the GIL) and collect reference-shaped results; the batching, the
    device work and the completion run in libarmi's own threads on the server's HIP stream.
    search_type "dense" answers every query by the dense branch of QdrantRetriever.search
    (qdrant.py:316-323); "hybrid" (a hybrid collection) answers a query that carries sparse
    terms by the hybrid branch (qdrant.py:272-298: prefetch 2k + 2k, RRF, hit.score = the RRF
    score) and one without by the dense branch, as search() chooses; "sparse" answers a query
    with terms by the sparse-only branch (qdrant.py:299-311: sparse top-k, hit.score = the dot).
    submit() takes a per-query search_type and filter_metadata as search() does: the filter is
    the collection's device row bitmask (ChunkCollection.filter_mask), held by the server until
    the ticket's result is read; the native server batches queries of one filter together.

    Lifetime: the collection knows its open servers and closes them before it frees its device
    indexes (ChunkCollection.close: delete_collection, load_collection, attach_collection); close()
    stops the native server, waits for the callers still inside it, then destroys it."""

    def __init__(self, retriever: MI355XRetriever, collection_name: str | None = None,
                 top_k: int | None = None, max_batch: int = 64, max_wait_ms: float = 2.0,
                 search_type: str = "dense"):
        from audio_rag_amd import _armi

        if search_type not in ("dense", "hybrid", "sparse"):
            raise ValueError("StreamServer search_type must be 'dense', 'hybrid' or 'sparse'")
        self.search_type = search_type
        self._armi = _armi
        self.retriever = retriever
        self.resolved = retriever._resolve_collection(collection_name)
        self.collection = retriever._collections[self.resolved]
        self.index = self.collection.dense_index  # kept alive for the server's lifetime
        self.sparse_index = self.collection.sparse_index if search_type != "dense" else None
        self.hybrid = self.sparse_index is not None
        self.k = top_k or retriever.config.top_k
        self.dim = retriever.embedding_dim
        self._handle = _armi.ctypes.c_void_p()
        self._lock = threading.Lock()
        self._idle = threading.Condition(self._lock)
        self._inflight = 0
        self._closed = False
        self._masks: dict[int, torch.Tensor] = {}  # ticket -> row filter the batch still reads
        if self.hybrid:
            _armi.call("armi_stream_create_hybrid", self.index.handle, self.sparse_index.handle,
                       self.k, retriever.config.rrf_k, max_batch, float(max_wait_ms) * 1e3,
                       _armi.ctypes.byref(self._handle))
        else:
            _armi.call("armi_stream_create", self.index.handle, self.k, max_batch,
                       float(max_wait_ms) * 1e3, _armi.ctypes.byref(self._handle))
        self.collection.attach_server(self)
        # QdrantRetriever.search applies score_threshold to legacy dense-only collections only
        # (qdrant.py:331), as MI355XRetriever.search does
        thr = retriever.config.score_threshold
        self.threshold = thr if (not self.collection.hybrid and thr > 0) else None

    def _call(self, fn: str, *args):
        """One native call on the live server (refused once close() has begun)."""
        with self._lock:
            if self._closed:
                raise RetrievalError("StreamServer is closed")
            self._inflight += 1
            h = self._handle
        try:
            return self._armi.call(fn, h, *args)
        except self._armi.ArmiError as e:  # retriever failures surface as RetrievalError
            raise RetrievalError(str(e)) from e
        finally:
            with self._lock:
                self._inflight -= 1
                if self._inflight == 0:
                    self._idle.notify_all()

    # QdrantRetriever.search's branch per search_type (qdrant.py:272-332): native mode codes
    _MODES = {"hybrid": 0, "dense": 1, "sparse": 2}  # ARMI_STREAM_AUTO / _DENSE / _SPARSE

    def submit_arrays(self, dense: np.ndarray,
                      sparse: tuple[np.ndarray, np.ndarray] | None = None,
                      filter_metadata: dict | None = None, search_type: str | None = None) -> int:
        """dense: [dim] query; sparse: (indices, values) or None; filter_metadata / search_type
        as MI355XRetriever.search (search_type None = the server's). Returns a ticket."""
        q = np.ascontiguousarray(dense, dtype=np.float16).reshape(-1)
        if q.size != self.dim:
            raise RetrievalError(f"query has {q.size} components, the store {self.dim}")
        st = search_type or self.search_type
        if st not in self._MODES:
            raise RetrievalError(f"unknown search_type {st!r}")
        # a query carrying a sparse vector, even an empty one, takes the hybrid / sparse-only
        # branch as search() does (`sparse is not None`; the reference's `if query.sparse` is
        # true for any SparseVector object, qdrant.py:272/299). The sparse lists exist only on a
        # hybrid collection (else search() takes the dense branch whatever search_type says)
        wants_sparse = st != "dense" and sparse is not None and self.collection.hybrid
        if wants_sparse and not self.hybrid:
            raise RetrievalError(f"search_type {st!r} needs a server created with search_type "
                                 "'hybrid' or 'sparse'")
        idx = val = None
        nnz = 0
        if wants_sparse:
            idx, val = _sorted_terms(*sparse)
            if idx.size > 256:
                raise RetrievalError("a sparse query may hold at most 256 terms")
            nnz = idx.size
            if nnz == 0:  # non-null arrays mark "has a (empty) sparse vector" for the server
                idx, val = np.zeros(1, dtype=np.int32), np.zeros(1, dtype=np.float32)
        mask = self.collection.filter_mask(filter_metadata)
        ticket = self._armi.ctypes.c_int64()
        self._call("armi_stream_submit_ex", q.ctypes.data,
                   None if idx is None else idx.ctypes.data,
                   None if val is None else val.ctypes.data, nnz,
                   self._MODES[st] if wants_sparse else 1,
                   None if mask is None else mask.data_ptr(), self._armi.ctypes.byref(ticket))
        if mask is not None:
            with self._lock:
                self._masks[ticket.value] = mask
        return ticket.value

    def submit(self, query: EmbeddingResult, filter_metadata: dict | None = None,
               search_type: str | None = None) -> int:
        return self.submit_arrays(np.asarray(query.dense, dtype=np.float32),
                                  query_sparse_arrays(query.sparse), filter_metadata, search_type)

    def raw_result(self, ticket: int, timeout: float = 60.0):
        """(scores [k] (fp64 RRF scores on the hybrid branch, else float32 cosine / sparse
        dot), ids int64 [k], count) of a ticket."""
        scores = np.empty(self.k, dtype=np.float32)
        rank = np.empty(self.k, dtype=np.float64)
        ids = np.empty(self.k, dtype=np.int64)
        count = self._armi.ctypes.c_int32()
        mode = self._armi.ctypes.c_int32()
        try:
            self._call("armi_stream_wait", ticket, scores.ctypes.data, ids.ctypes.data,
                       rank.ctypes.data, self._armi.ctypes.byref(count),
                       self._armi.ctypes.byref(mode), timeout * 1e6)
        finally:
            with self._lock:
                self._masks.pop(ticket, None)
        return (rank if mode.value == 1 else scores), ids, count.value

    def result(self, ticket: int, timeout: float = 60.0) -> list[RetrievalResult]:
        """The ticket's list[RetrievalResult] (as MI355XRetriever.search builds it)."""
        from audio_rag_amd.core.base import AudioChunk

        scores, ids, c = self.raw_result(ticket, timeout)
        out = []
        for pid, score in zip(ids[:c].tolist(), scores[:c].tolist()):
            if self.threshold is not None and score < self.threshold:
                continue
            p = self.collection.payloads[pid]
            chunk = AudioChunk(text=p.get("text", ""), start=p.get("start", 0.0),
                               end=p.get("end", 0.0), speaker=p.get("speaker"),
                               metadata=p.get("metadata"))
            out.append(RetrievalResult(chunk=chunk, score=float(score), source=self.resolved))
        return out

    def search(self, query: EmbeddingResult, filter_metadata: dict | None = None,
               search_type: str | None = None) -> list[RetrievalResult]:
        return self.result(self.submit(query, filter_metadata, search_type))

    def stats(self) -> tuple[int, int]:
        b, q = self._armi.ctypes.c_int64(), self._armi.ctypes.c_int64()
        self._call("armi_stream_stats", self._armi.ctypes.byref(b), self._armi.ctypes.byref(q))
        return b.value, q.value

    def loadgen(self, queries: np.ndarray, n_queries: int, qps: float, seed: int = 0,
                sparse_csr: tuple[np.ndarray, np.ndarray, np.ndarray] | None = None,
                answers: bool = False):
        """Native open-loop Poisson load at `qps` (armi_stream_loadgen): query i = row
        (i % len(queries)) with, on a hybrid server, the terms of CSR row (i % len(queries)).
        Returns per-query latency in seconds and the elapsed time from the first submit to the
        last completion; with answers=True also every query's ids [n_queries, k] and count."""
        q = np.ascontiguousarray(queries, dtype=np.float16).reshape(-1, self.dim)
        lat = np.empty(n_queries, dtype=np.float64)
        el = self._armi.ctypes.c_double()
        done = self._armi.ctypes.c_int64()
        ptrs = (None, None, None)
        keep = None
        if sparse_csr is not None and self.hybrid:
            keep = _sorted_csr(*sparse_csr)
            if keep[0].size != q.shape[0] + 1:
                raise ValueError("one CSR row per query vector is required")
            if np.diff(keep[0]).max(initial=0) > 256:
                raise RetrievalError("a sparse query may hold at most 256 terms")
            ptrs = tuple(a.ctypes.data for a in keep)
        ids = np.empty((n_queries, self.k), dtype=np.int64) if answers else None
        cnt = np.empty(n_queries, dtype=np.int32) if answers else None
        self._call("armi_stream_loadgen", q.ctypes.data, *ptrs, q.shape[0], n_queries,
                   float(qps), seed, lat.ctypes.data, self._armi.ctypes.byref(el),
                   self._armi.ctypes.byref(done), None if ids is None else ids.ctypes.data,
                   None if cnt is None else cnt.ctypes.data)
        if answers:
            return lat * 1e-6, el.value, ids, cnt
        return lat * 1e-6, el.value

    def close(self) -> None:
        with self._lock:
            if self._closed:
                return
            self._closed = True
            h = self._handle
        if h and h.value:
            # wake every caller blocked inside the server, let them leave, then free it
            self._armi.call("armi_stream_stop", h)
            with self._lock:
                while self._inflight:
                    self._idle.wait()
            self._armi.call("armi_stream_destroy", h)
        self._handle = self._armi.ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
