"""Device-side chunk-store handles over libarmi (torch tensors in, torch tensors out).

Everything here runs on the GPU through the C ABI in include/armi.h; torch only provides device
memory and the stream. Results stay on the device until the caller materialises them.
"""

from __future__ import annotations

import ctypes

import torch

from audio_rag_amd import _armi
from audio_rag_amd._armi import call, ptr, query, stream_handle

MAX_K = 240
QUERY_BLOCK = 64  # queries per scan pass of armi_dense_topk


class TopK:
    """Per-query top-k on the device. ids are chunk ordinals (-1 past count).

    scores  float32 [B, k]
    ids     int64   [B, k]
    rank    float64 [B, k] ranking key (dense: the exact cosine key; sparse: the scores; fused
            lists: the RRF score)
    count   int32   [B]
    flags   int32   [B] ARMI_FLAG_* bits, or None

    A list whose kernel writes only one of scores / rank gets the other converted on first access
    (on the stream current then), so a hybrid step that reads neither launches no conversion."""

    __slots__ = ("_scores", "ids", "_rank", "count", "flags")

    def __init__(self, scores=None, ids=None, rank=None, count=None, flags=None):
        self._scores, self.ids, self._rank, self.count, self.flags = scores, ids, rank, count, flags

    @property
    def scores(self) -> torch.Tensor | None:
        if self._scores is None and self._rank is not None:
            self._scores = self._rank.float()
        return self._scores

    @scores.setter
    def scores(self, t) -> None:
        self._scores = t

    @property
    def rank(self) -> torch.Tensor | None:
        if self._rank is None and self._scores is not None:
            self._rank = self._scores.double()
        return self._rank

    @rank.setter
    def rank(self, t) -> None:
        self._rank = t

    def tensors(self) -> tuple:
        """The device tensors this list holds now (no lazy conversion)."""
        return tuple(t for t in (self._scores, self.ids, self._rank, self.count, self.flags)
                     if t is not None)


def _check_fp16_2d(t: torch.Tensor, name: str, dim: int | None = None) -> None:
    if not isinstance(t, torch.Tensor) or t.dtype != torch.float16 or t.dim() != 2:
        raise ValueError(f"{name} must be a 2-D float16 tensor")
    if not t.is_cuda:
        raise ValueError(f"{name} must live on the GPU")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if dim is not None and t.shape[1] != dim:
        raise ValueError(f"{name} has dim {t.shape[1]}, index has {dim}")


class DenseIndex:
    """The Qdrant named vector "dense" (VectorParams(size=dim, distance=COSINE)) of
    src/audio_rag/retrieval/qdrant.py:93-109, as an fp16 row store in HBM.

    rows: [N, dim] float16 on the device (kept alive by this object)."""

    def __init__(self, rows: torch.Tensor, ordinal_base: int = 0):
        _check_fp16_2d(rows, "rows")
        self.rows = rows
        self.dim = int(rows.shape[1])
        self.n_rows = int(rows.shape[0])
        self.ordinal_base = int(ordinal_base)
        self.device = rows.device
        self._handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            call("armi_index_create", self.device.index or 0, ptr(rows), self.n_rows, self.dim,
                 self.ordinal_base, ctypes.byref(self._handle), stream_handle())

    def close(self) -> None:
        if self._handle and self._handle.value:
            torch.cuda.synchronize(self.device)
            _armi.call("armi_index_destroy", self._handle)
            self._handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._handle

    def invalid_rows(self) -> int:
        torch.cuda.current_stream(self.device).synchronize()
        return int(query("armi_index_invalid_rows", self._handle))

    def norms(self) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """(norm2 int64, inv_norm float64, inv_norm32 float32) copies of the index's arrays."""
        p2, pi, p32 = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        call("armi_index_norms", self._handle, ctypes.byref(p2), ctypes.byref(pi), ctypes.byref(p32))
        n = self.n_rows
        out = (torch.empty(n, dtype=torch.int64, device=self.device),
               torch.empty(n, dtype=torch.float64, device=self.device),
               torch.empty(n, dtype=torch.float32, device=self.device))
        torch.cuda.current_stream(self.device).synchronize()
        for src, dst in zip((p2, pi, p32), out):
            _device_copy(dst.data_ptr(), src.value, dst.numel() * dst.element_size())
        return out

    def scan_form(self, n_queries: int, k: int) -> int:
        """Which scan armi_dense_topk runs for this call shape (_armi.SCAN_*)."""
        return int(query("armi_dense_scan_form", self._handle, n_queries, k))

    def scan_nontemporal(self, n_queries: int, k: int) -> bool:
        """Whether the int8 first pass of this call shape streams with nontemporal loads."""
        return int(query("armi_dense_scan_nontemporal", self._handle, n_queries, k)) == 1

    def workspace_bytes(self, n_queries: int, k: int, exact: bool = False) -> int:
        fn = "armi_dense_exact_workspace_bytes" if exact else "armi_dense_workspace_bytes"
        return int(query(fn, self._handle, n_queries, k))

    def topk(self, queries: torch.Tensor, k: int, row_mask: torch.Tensor | None = None,
             exact: bool = False, workspace: torch.Tensor | None = None,
             out: TopK | None = None) -> TopK:
        """Cosine top-k of every query row. row_mask: int64 tensor holding a bitmask of enabled
        rows (bit r of word r // 64), or None."""
        _check_fp16_2d(queries, "queries", self.dim)
        if not 1 <= k <= MAX_K:
            raise ValueError(f"k must be in [1, {MAX_K}]")
        b = int(queries.shape[0])
        dev = self.device
        if row_mask is not None:
            need = (self.n_rows + 63) // 64
            if row_mask.dtype != torch.int64 or row_mask.numel() < need or not row_mask.is_cuda:
                raise ValueError(f"row_mask must be an int64 device tensor of >= {need} words")
        if out is None:
            out = TopK(scores=torch.empty((b, k), dtype=torch.float32, device=dev),
                       ids=torch.empty((b, k), dtype=torch.int64, device=dev),
                       rank=torch.empty((b, k), dtype=torch.float64, device=dev),
                       count=torch.empty(b, dtype=torch.int32, device=dev),
                       flags=torch.empty(b, dtype=torch.int32, device=dev))
        need = self.workspace_bytes(max(b, 1), k, exact)
        if workspace is None or workspace.numel() < need:
            workspace = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
        s = stream_handle()
        if exact:
            call("armi_dense_exact_topk", self._handle, ptr(queries), b, k, ptr(row_mask),
                 ptr(out.scores), ptr(out.ids), ptr(out.rank), ptr(out.count), ptr(workspace),
                 workspace.numel(), s)
            if out.flags is not None:
                out.flags.fill_(_armi.ARMI_FLAG_FALLBACK)
        else:
            call("armi_dense_topk", self._handle, ptr(queries), b, k, ptr(row_mask),
                 ptr(out.scores), ptr(out.ids), ptr(out.rank), ptr(out.count), ptr(out.flags),
                 ptr(workspace), workspace.numel(), s)
        return out


class SparseIndex:
    """The Qdrant sparse vector "sparse" (SparseVectorParams(index=SparseIndexParams(on_disk=
    False)), no IDF modifier) of src/audio_rag/retrieval/qdrant.py:103-107, as a CSR in HBM.

    indptr int64 [N+1], indices int32 (ascending within a row), values float32; device tensors
    kept alive by this object."""

    def __init__(self, indptr: torch.Tensor, indices: torch.Tensor, values: torch.Tensor,
                 vocab: int, ordinal_base: int = 0):
        for t, dt, name in ((indptr, torch.int64, "indptr"), (indices, torch.int32, "indices"),
                            (values, torch.float32, "values")):
            if t.dtype != dt or t.dim() != 1 or not t.is_cuda or not t.is_contiguous():
                raise ValueError(f"{name} must be a contiguous 1-D {dt} device tensor")
        self.indptr, self.indices, self.values = indptr, indices, values
        self.n_rows = int(indptr.numel()) - 1
        self.vocab = int(vocab)
        self.ordinal_base = int(ordinal_base)
        self.device = indptr.device
        self._handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            call("armi_sparse_index_create", self.device.index or 0, ptr(indptr), ptr(indices),
                 ptr(values), self.n_rows, int(indices.numel()), self.vocab, self.ordinal_base,
                 ctypes.byref(self._handle), stream_handle())

    def close(self) -> None:
        if self._handle and self._handle.value:
            torch.cuda.synchronize(self.device)
            _armi.call("armi_sparse_index_destroy", self._handle)
            self._handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._handle

    def workspace_bytes(self, n_queries: int, k: int) -> int:
        return int(query("armi_sparse_workspace_bytes", self._handle, n_queries, k))

    def set_filter(self, enable: bool) -> bool:
        """Turns armi_sparse_topk's MFMA filter on / off (on by default; off = the exact scan
        alone, the same results); returns whether the index can use it (every value >= 0)."""
        usable = ctypes.c_int()
        torch.cuda.current_stream(self.device).synchronize()
        call("armi_sparse_index_set_filter", self._handle, int(bool(enable)), ctypes.byref(usable))
        return bool(usable.value)

    def topk(self, q_indptr: torch.Tensor, q_indices: torch.Tensor, q_values: torch.Tensor, k: int,
             row_mask: torch.Tensor | None = None, workspace: torch.Tensor | None = None) -> TopK:
        """Sparse dot top-k for a query CSR (q_indptr int32 [B+1], ascending q_indices int32,
        q_values float32, all on the device)."""
        if not 1 <= k <= MAX_K:
            raise ValueError(f"k must be in [1, {MAX_K}]")
        b = int(q_indptr.numel()) - 1
        dev = self.device
        out = TopK(scores=torch.empty((b, k), dtype=torch.float32, device=dev),
                   ids=torch.empty((b, k), dtype=torch.int64, device=dev),
                   count=torch.empty(b, dtype=torch.int32, device=dev),
                   flags=torch.empty(b, dtype=torch.int32, device=dev))
        if b == 0:
            return out
        need = self.workspace_bytes(b, k)
        if workspace is None or workspace.numel() < need:
            workspace = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
        call("armi_sparse_topk", self._handle, ptr(q_indptr), ptr(q_indices), ptr(q_values), b, k,
             ptr(row_mask), ptr(out.scores), ptr(out.ids), ptr(out.count), ptr(out.flags),
             ptr(workspace), workspace.numel(), stream_handle())
        return out


def merge_shards(rank: torch.Tensor, scores: torch.Tensor, ids: torch.Tensor, count: torch.Tensor,
                 k_out: int) -> TopK:
    """Global top-k from per-shard lists [S, B, k_in] (+ count [S, B]) gathered from all ranks."""
    s, b, k_in = ids.shape
    dev = ids.device
    out = TopK(scores=torch.empty((b, k_out), dtype=torch.float32, device=dev),
               ids=torch.empty((b, k_out), dtype=torch.int64, device=dev),
               rank=torch.empty((b, k_out), dtype=torch.float64, device=dev),
               count=torch.empty(b, dtype=torch.int32, device=dev))
    # hold the contiguous copies until the launch is enqueued (a freed temporary's block can be
    # handed to the next allocation before the kernel reads it)
    rank, scores, ids, count = (t.contiguous() for t in (rank, scores, ids, count))
    call("armi_topk_merge_shards", ptr(rank), ptr(scores), ptr(ids), ptr(count), s, b, k_in,
         k_out, ptr(out.rank), ptr(out.scores), ptr(out.ids), ptr(out.count), stream_handle())
    return out


def merge_shards_packed(buf: torch.Tensor, row0: int, n_queries: int, offsets: tuple[int, int, int, int],
                        k_in: int, k_out: int) -> TopK:
    """merge_shards over the all-gathered exchange buffer in place: buf uint8 [S, rows, W] (one
    byte row per (shard, query), shards.pack_rows' layout), this rank's queries at rows
    [row0, row0 + n_queries); offsets = byte offsets of (rank f64, scores f32, ids i64, count i32)
    inside a row. One launch, no per-field copies (armi_topk_merge_shards_packed)."""
    s, rows, w = buf.shape
    if not buf.is_contiguous():
        raise ValueError("merge_shards_packed: the exchange buffer must be contiguous")
    dev = buf.device
    out = TopK(scores=torch.empty((n_queries, k_out), dtype=torch.float32, device=dev),
               ids=torch.empty((n_queries, k_out), dtype=torch.int64, device=dev),
               rank=torch.empty((n_queries, k_out), dtype=torch.float64, device=dev),
               count=torch.empty(n_queries, dtype=torch.int32, device=dev))
    off_rank, off_scores, off_ids, off_count = offsets
    call("armi_topk_merge_shards_packed", buf.data_ptr() + row0 * w, rows * w, w, off_rank,
         off_scores, off_ids, off_count, s, n_queries, k_in, k_out, ptr(out.rank),
         ptr(out.scores), ptr(out.ids), ptr(out.count), stream_handle())
    return out


def rrf_fuse(a: TopK, b: TopK, limit: int, rrf_k: int = 2) -> TopK:
    """FusionQuery(RRF) of two prefetch lists (qdrant.py:295). rank/scores hold the fp64 RRF
    score (scores as float32 for convenience)."""
    n, ka = a.ids.shape
    kb = b.ids.shape[1]
    dev = a.ids.device
    out_ids = torch.empty((n, limit), dtype=torch.int64, device=dev)
    out_score = torch.empty((n, limit), dtype=torch.float64, device=dev)
    out_count = torch.empty(n, dtype=torch.int32, device=dev)
    a_ids, b_ids = a.ids.contiguous(), b.ids.contiguous()
    a_cnt, b_cnt = a.count.to(torch.int32).contiguous(), b.count.to(torch.int32).contiguous()
    call("armi_rrf_fuse", ptr(a_ids), ptr(a_cnt), ka, ptr(b_ids), ptr(b_cnt), kb, n, rrf_k, limit,
         ptr(out_ids), ptr(out_score), ptr(out_count), stream_handle())
    return TopK(ids=out_ids, rank=out_score, count=out_count)


class ConcurrentHybrid:
    """The two prefetches of one hybrid search (qdrant.py:281-298) on two HIP streams: the
    sparse top-k on a side stream, the dense scan and merge on the caller's stream (the two share
    nothing until the fusion), then RRF on the caller's stream. The two scans cannot share a CU
    (each fills its LDS and register file), so in a kernel trace they run nearly one after the
    other (profiles/r05m_hybrid_kernel_stats.csv); what overlaps is the small kernels
    of one chain (merges, collect passes, pass_terms) with the other chain's scan and tail: both
    chains on one stream measured 0.550 against 0.522 ms per step on one box (r05t)."""

    def __init__(self, device: torch.device):
        self.side = torch.cuda.Stream(device=device)

    def __call__(self, dense_fn, sparse_fn, sparse_inputs, limit: int, rrf_k: int = 2) -> TopK:
        main = torch.cuda.current_stream()
        self.side.wait_stream(main)
        # (under graph capture the graph's pool owns every block: no cross-stream bookkeeping)
        capturing = torch.cuda.is_current_stream_capturing()
        for t in sparse_inputs:
            if isinstance(t, torch.Tensor) and t.is_cuda and not capturing:
                t.record_stream(self.side)
        # the sparse chain is issued first (round-3 A/B: profiles/r03x_*)
        with torch.cuda.stream(self.side):
            s = sparse_fn()
        d = dense_fn()
        main.wait_stream(self.side)
        if not capturing:
            for t in s.tensors():
                t.record_stream(main)
        return rrf_fuse(d, s, limit, rrf_k=rrf_k)


_hip = None


def _device_copy(dst: int, src: int, nbytes: int) -> None:
    """Synchronous device-to-device copy through the process's HIP runtime (the one torch
    loaded), for reading the index's internal arrays in tests."""
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so.7")
        _hip.hipMemcpy.restype = ctypes.c_int
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    rc = _hip.hipMemcpy(ctypes.c_void_p(dst), ctypes.c_void_p(src), nbytes, 3)  # DeviceToDevice
    if rc != 0:
        raise RuntimeError(f"hipMemcpy failed: {rc}")


class HybridGraph:
    """One hybrid step over a fixed batch size (ConcurrentHybrid: dense top-k, sparse top-k, RRF)
    captured as a HIP graph. The step's inputs live in one staging buffer (fp16 queries, query
    CSR indptr / indices / values at fixed offsets): a call copies a batch into it, one copy for
    a batch prepared by pack() (or one per array), and replays every kernel of the step. The
    eager step's ~20 launches with their Python argument handling take longer on the host than
    the step takes on the GPU, so eager steps leave the GPU idle between them (30 us per 0.54 ms
    step in profiles/r05m_hybrid_kernel_stats.csv's trace).

    The returned TopK's tensors are the graph's outputs: a later call overwrites them, so callers
    consume (or clone) a result before the next call."""

    def __init__(self, dense: DenseIndex, sparse: SparseIndex, batch: int, pre_k: int, limit: int,
                 rrf_k: int = 2, max_terms: int = 256):
        dev = dense.device
        self.batch, self.dim, self.max_terms = int(batch), dense.dim, int(max_terms)
        self._off = self._layout(self.batch, self.dim, self.max_terms)
        self.stage = torch.zeros(self._off[-1], dtype=torch.uint8, device=dev)
        self.q, self.qi, self.qx, self.qv = self._views(self.stage)
        ws = torch.empty(max(dense.workspace_bytes(batch, pre_k), 1), dtype=torch.uint8, device=dev)
        sws = torch.empty(max(sparse.workspace_bytes(batch, pre_k), 1), dtype=torch.uint8,
                          device=dev)
        hybrid = ConcurrentHybrid(dev)

        def run() -> TopK:
            return hybrid(lambda: dense.topk(self.q, pre_k, workspace=ws),
                          lambda: sparse.topk(self.qi, self.qx, self.qv, pre_k, workspace=sws),
                          (self.qi, self.qx, self.qv), limit, rrf_k)

        # warm-up on a side stream, then capture under inference mode (as _QueryGraph and the
        # reranker's graphs do: the CUDA generator's graph state is shared by every capture).
        # The warm-up batch is one-hot dense queries with empty sparse parts: all-zero queries
        # tie every row at cosine 0, so their top-k cannot be certified and the warm-up ran the
        # dense collect pass over the whole shard (~0.16 s per call at 1M rows, r05z trace)
        rows = torch.arange(self.batch, device=dev)
        self.q[rows, rows % self.dim] = 1.0
        with torch.inference_mode():
            side = torch.cuda.Stream(device=dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(2):
                    run()
            torch.cuda.current_stream(dev).wait_stream(side)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.out = run()
        self._keep = (ws, sws, hybrid, dense, sparse)

    @staticmethod
    def _layout(batch: int, dim: int, max_terms: int) -> tuple[int, int, int, int, int]:
        def up(x: int) -> int:
            return (x + 255) // 256 * 256

        o_qi = up(batch * dim * 2)
        o_qx = o_qi + up((batch + 1) * 4)
        o_qv = o_qx + up(batch * max_terms * 4)
        return 0, o_qi, o_qx, o_qv, o_qv + up(batch * max_terms * 4)

    def _views(self, buf: torch.Tensor):
        o_q, o_qi, o_qx, o_qv, end = self._off
        b, n = self.batch, self.batch * self.max_terms
        return (buf[o_q:o_qi].view(torch.float16)[: b * self.dim].view(b, self.dim),
                buf[o_qi:o_qx].view(torch.int32)[: b + 1], buf[o_qx:o_qv].view(torch.int32)[:n],
                buf[o_qv:end].view(torch.float32)[:n])

    def _check(self, queries, q_indptr, q_indices, q_values) -> int:
        """Shape checks of a batch. The per-query limit of max_terms (armi_sparse_topk scores a
        longer query's first 256 terms only and flags it) is checked here for a host indptr; a
        device indptr is not read back (that would synchronise every step): callers keep each
        query within max_terms, as query_sparse_arrays does for the pipeline."""
        n = int(q_indices.numel())
        if (tuple(queries.shape) != (self.batch, self.dim) or int(q_indptr.numel()) != self.batch + 1
                or n > self.batch * self.max_terms or int(q_values.numel()) != n):
            raise ValueError("HybridGraph: batch shape differs from the captured one")
        if not q_indptr.is_cuda and self.batch > 0:
            lens = q_indptr[1:].to(torch.int64) - q_indptr[:-1].to(torch.int64)
            if int(lens.max()) > self.max_terms or int(lens.min()) < 0:
                raise ValueError(f"HybridGraph: a query has more than {self.max_terms} terms")
        return n

    def pack(self, queries: torch.Tensor, q_indptr: torch.Tensor, q_indices: torch.Tensor,
             q_values: torch.Tensor) -> torch.Tensor:
        """A batch in the staging layout (one device buffer), for __call__(packed)."""
        n = self._check(queries, q_indptr, q_indices, q_values)
        buf = torch.zeros_like(self.stage)
        q, qi, qx, qv = self._views(buf)
        q.copy_(queries)
        qi.copy_(q_indptr)
        qx[:n].copy_(q_indices)
        qv[:n].copy_(q_values)
        return buf

    def __call__(self, *batch: torch.Tensor) -> TopK:
        """hg(packed) with a pack() buffer (one copy), or hg(queries, q_indptr, q_indices,
        q_values)."""
        if len(batch) == 1:
            if batch[0].shape != self.stage.shape or batch[0].dtype != torch.uint8:
                raise ValueError("HybridGraph: not a pack() buffer of this graph")
            self.stage.copy_(batch[0])
        else:
            queries, q_indptr, q_indices, q_values = batch
            n = self._check(queries, q_indptr, q_indices, q_values)
            self.q.copy_(queries)
            self.qi.copy_(q_indptr)
            self.qx[:n].copy_(q_indices)
            self.qv[:n].copy_(q_values)
        self.graph.replay()
        return self.out
