"""Corpus sharded by chunk ordinal over the GPUs of one node (one process per GPU).

No reference counterpart: the reference runs a single Qdrant replica
(k8s/helm/audio-rag/values.yaml:137) and scales API processes (Dockerfile.api:85-86). Sharding
is exact for this path because every ranking key is comparable across shards (dense: exact
cosine key; sparse: exact fp32 score; both tie-broken by the global ordinal), so the global top-k
is the top-k of the union of per-shard top-k lists.

One search step for a process group of G ranks, each bringing B queries:
  1. all-gather the queries (RCCL over xGMI): every rank holds all G*B queries. Dense rows and,
     for hybrid / sparse search, the sparse query terms travel in ONE collective: each query's
     terms are padded to MAX_QUERY_TERMS fixed slots, so the message size is known on every rank
     without a host round trip.
  2. local top-k of all G*B queries on this rank's shard (libarmi kernels); for hybrid the dense
     scan runs on the caller's stream and the sparse scan on a side stream, concurrently.
  3. all-gather the per-shard lists (dense and sparse together for hybrid), packed into one byte
     buffer per query: one collective.
  4. merge this rank's B queries over the G shard lists (armi_topk_merge_shards), then RRF for
     hybrid.
Nothing in a step waits on the host: no .item() / .tolist(), so the whole step is enqueued
asynchronously. Per-GPU work is fixed as G grows (shard rows x G*B queries = corpus x B): weak
scaling.
"""

from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist

from audio_rag_amd._armi import call, ptr, stream_handle
from audio_rag_amd.retrieval.device import TopK

MAX_QUERY_TERMS = 256  # armi_sparse_topk's per-query term capacity (include/armi.h)

LocalSearch = Callable[[torch.Tensor, int], TopK]
Merge = Callable[[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, int], TopK]


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous ordinal range [lo, hi) owned by `rank` (rank r owns [r*n/G, (r+1)*n/G))."""
    return n * rank // world, n * (rank + 1) // world


def _all_gather(out: torch.Tensor, inp: torch.Tensor, group) -> None:
    """out: [G, *inp.shape]. RCCL gathers straight into the tensor; gloo (CPU tests) into views."""
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, inp, group=group)
    else:
        dist.all_gather(list(out.unbind(0)), inp, group=group)


def _bytes(t: torch.Tensor, n: int) -> torch.Tensor:
    """[n, ...] tensor -> its bytes as uint8 [n, row_bytes]."""
    return t.contiguous().reshape(n, -1).view(torch.uint8)


def pack_rows(parts: list[torch.Tensor]) -> tuple[torch.Tensor, list[tuple[int, int, torch.dtype, tuple]]]:
    """Concatenates per-query tensors (leading dim n) into one uint8 [n, bytes] buffer; returns it
    with the layout unpack_rows needs. Parts are laid out by element size, largest first, so every
    part starts at a multiple of its own element size: a one-row slice of the buffer (contiguous,
    so not copied by unpack_rows) can be viewed as its dtype in place."""
    n = int(parts[0].shape[0])
    order = sorted(range(len(parts)), key=lambda i: -parts[i].element_size())
    layout, off = [None] * len(parts), 0
    for i in order:
        nbytes = int(_bytes(parts[i], n).shape[1])
        layout[i] = (off, nbytes, parts[i].dtype, tuple(parts[i].shape[1:]))
        off += nbytes
    cols = [_bytes(parts[i], n) for i in order]
    if off % 8:  # rows a multiple of 8 bytes: every row's fields stay naturally aligned
        cols.append(torch.empty((n, 8 - off % 8), dtype=torch.uint8, device=parts[0].device))
    return torch.cat(cols, dim=1), layout


def unpack_rows(buf: torch.Tensor, layout) -> list[torch.Tensor]:
    """Inverse of pack_rows on a buffer [..., bytes]: tensors [..., *shape] of the packed dtypes,
    in the order pack_rows received them."""
    lead = tuple(buf.shape[:-1])
    return [buf[..., off:off + nbytes].contiguous().view(dtype).reshape(lead + shape)
            for off, nbytes, dtype, shape in layout]


def pad_csr(indptr: torch.Tensor, idx: torch.Tensor, val: torch.Tensor,
            slots: int = MAX_QUERY_TERMS) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """CSR (indptr [n+1], indices, values) -> fixed slots (count int32 [n], indices int32 [n, slots],
    values float32 [n, slots]) without a host synchronisation. GPU tensors: one libarmi launch
    (armi_query_slots_pack); host tensors (the gloo CPU tests' exchange): torch ops."""
    n = int(indptr.numel()) - 1
    dev = indptr.device
    if indptr.is_cuda:
        count = torch.empty(n, dtype=torch.int32, device=dev)
        pi = torch.empty((n, slots), dtype=torch.int32, device=dev)
        pv = torch.empty((n, slots), dtype=torch.float32, device=dev)
        ip32, i32, v32 = (t.to(d).contiguous() for t, d in
                          ((indptr, torch.int32), (idx, torch.int32), (val, torch.float32)))
        call("armi_query_slots_pack", ptr(ip32), ptr(i32), ptr(v32), n, slots, ptr(count),
             ptr(pi), ptr(pv), stream_handle())
        return count, pi, pv
    ip = indptr.to(torch.int64)
    # callers refuse queries longer than `slots` up front (query_sparse_arrays raises); the
    # clamp only keeps the padded CSR self-consistent without a host synchronisation
    count = (ip[1:] - ip[:-1]).clamp(max=slots).to(torch.int32)
    pi = torch.zeros(n * slots + 1, dtype=torch.int32, device=dev)
    pv = torch.zeros(n * slots + 1, dtype=torch.float32, device=dev)
    nnz = int(idx.numel())  # the tensor's size, known on the host
    if nnz and n:
        e = torch.arange(nnz, dtype=torch.int64, device=dev)
        # query owning element e; entries past indptr[-1] (a CSR may carry unused trailing
        # entries, e.g. the first rows of a larger query batch) and terms past a query's `slots`
        # go to the dump slot n * slots, so no write lands outside the buffers
        q = torch.searchsorted(ip[1:], e, right=True).clamp_(max=n - 1)
        j = e - ip[q]
        pos = torch.where((e < ip[n]) & (j < slots), q * slots + j, torch.full_like(e, n * slots))
        pi.index_copy_(0, pos, idx.to(torch.int32))
        pv.index_copy_(0, pos, val.to(torch.float32))
    return count, pi[:-1].view(n, slots), pv[:-1].view(n, slots)


def unpad_csr(count: torch.Tensor, pi: torch.Tensor, pv: torch.Tensor):
    """Inverse of pad_csr: (indptr int32 [n+1], indices, values). The index / value arrays keep
    their padded length; entries past indptr[-1] are unused (the CSR ends at indptr[-1])."""
    n, slots = pi.shape
    dev = pi.device
    indptr = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(count.to(torch.int64), 0, out=indptr[1:])
    j = torch.arange(slots, dtype=torch.int64, device=dev)
    live = j[None, :] < count.to(torch.int64)[:, None]
    # live slot (q, j) -> indptr[q] + j; dead slots -> a dump slot past the end
    pos = torch.where(live, indptr[:-1, None] + j[None, :], torch.full_like(j[None, :], n * slots))
    oi = torch.zeros(n * slots + 1, dtype=torch.int32, device=dev)
    ov = torch.zeros(n * slots + 1, dtype=torch.float32, device=dev)
    oi.index_copy_(0, pos.reshape(-1), pi.reshape(-1))
    ov.index_copy_(0, pos.reshape(-1), pv.reshape(-1))
    return indptr.to(torch.int32), oi[:-1], ov[:-1]


def _topk_parts(t: TopK) -> list[torch.Tensor]:
    return [t.rank.to(torch.float64), t.ids, t.scores, t.count.to(torch.int32).view(-1, 1)]


class ShardedSearch:
    """Sharded top-k over a process group. `local_dense(q, k)` / `local_sparse(qcsr, k)` search
    this rank's shard and return global ordinals; `merge` combines [S, B, k] lists."""

    def __init__(self, local_dense: LocalSearch, merge: Merge, group=None,
                 local_sparse: Callable | None = None, rrf: Callable | None = None,
                 merge_packed: Callable | None = None):
        """merge_packed (device.merge_shards_packed): merges straight from the gathered byte
        buffer when it lives on the GPU; `merge` serves host buffers (the CPU tests)."""
        self.local_dense = local_dense
        self.local_sparse = local_sparse
        self.merge = merge
        self.merge_packed = merge_packed
        self.rrf = rrf
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self._side: torch.cuda.Stream | None = None
        # search(): gathered query rows that are real queries (None: all of them); the rest pad
        # a smaller batch to the largest one and are never scanned (_dense_local)
        self._live: torch.Tensor | None = None
        self.scanned_queries = 0  # dense queries this rank's last local scan searched
        self.last_dense_flags: torch.Tensor | None = None  # ARMI_FLAG_* of those queries

    # ------------------------------------------------------------------ collectives

    def _gather(self, buf: torch.Tensor) -> torch.Tensor:
        out = torch.empty((self.world,) + tuple(buf.shape), dtype=buf.dtype, device=buf.device)
        _all_gather(out, buf, self.group)
        return out

    def _gather_queries(self, q_dense: torch.Tensor | None, q_csr=None):
        """All queries of all ranks: (dense [G*nb, dim] or None, csr of G*nb queries or None)."""
        parts = []
        if q_dense is not None:
            parts.append(q_dense)
        if q_csr is not None:
            parts.extend(pad_csr(*q_csr))
        buf, layout = pack_rows(parts)
        g = self._gather(buf)                              # [G, nb, bytes]
        g = g.reshape((-1,) + tuple(g.shape[2:]))          # [G*nb, bytes]
        if g.is_cuda and q_csr is not None:
            # the CSR straight from the gathered rows (one launch, no per-field copies)
            dense = unpack_rows(g, layout[:1])[0] if q_dense is not None else None
            lc, li, lv = layout[-3:]
            n, slots = int(g.shape[0]), li[3][0]
            indptr = torch.empty(n + 1, dtype=torch.int32, device=g.device)
            idx = torch.empty(n * slots, dtype=torch.int32, device=g.device)
            val = torch.empty(n * slots, dtype=torch.float32, device=g.device)
            call("armi_query_slots_unpack", g.data_ptr(), int(g.stride(0)), lc[0], li[0], lv[0], n,
                 slots, ptr(indptr), ptr(idx), ptr(val), stream_handle())
            return dense, (indptr, idx, val)
        vals = unpack_rows(g, layout)
        dense = vals.pop(0) if q_dense is not None else None
        csr = unpad_csr(*vals) if q_csr is not None else None
        return dense, csr

    def _exchange(self, lists: list[TopK], k: int, nb: int) -> list[TopK]:
        """All-gathers per-shard lists of all G*nb queries (several searches in one message) and
        merges this rank's nb queries over the G shards."""
        parts = [p for t in lists for p in _topk_parts(t)]
        buf, layout = pack_rows(parts)
        g = self._gather(buf)                              # [G, G*nb, bytes]
        if self.merge_packed is not None and g.is_cuda:
            # each list's (rank, scores, ids, count) read in place from the gathered rows
            return [self.merge_packed(g, self.rank * nb, nb,
                                      tuple(layout[4 * i + j][0] for j in (0, 2, 1, 3)),
                                      layout[4 * i + 1][3][0], k)
                    for i in range(len(lists))]
        mine = g[:, self.rank * nb:(self.rank + 1) * nb]   # [G, nb, bytes]
        vals = unpack_rows(mine, layout)
        out = []
        for i in range(len(lists)):
            rank, ids, scores, count = vals[4 * i:4 * i + 4]
            out.append(self.merge(rank, scores, ids, count.reshape(count.shape[:2]), k))
        return out

    # ------------------------------------------------------------------------ search

    def gather_queries(self, q_local: torch.Tensor) -> torch.Tensor:
        return self._gather_queries(q_local)[0]

    def dense(self, q_local: torch.Tensor, k: int) -> TopK:
        nb = int(q_local.shape[0])
        all_q, _ = self._gather_queries(q_local)
        return self._exchange([self._dense_local(all_q, k)], k, nb)[0]

    def sparse(self, q_local_csr: tuple[torch.Tensor, torch.Tensor, torch.Tensor], k: int) -> TopK:
        """q_local_csr: (indptr int32 [nb+1], indices int32, values float32) of this rank."""
        nb = int(q_local_csr[0].numel()) - 1
        _, all_csr = self._gather_queries(None, q_local_csr)
        return self._exchange([self.local_sparse(all_csr, k)], k, nb)[0]

    def hybrid(self, q_local: torch.Tensor, q_local_csr, k: int) -> TopK:
        """Prefetch dense and sparse 2k each on the global corpus, then RRF(limit=k). One
        collective for the queries, the two local scans concurrent, one for the lists."""
        nb = int(q_local.shape[0])
        all_q, all_csr = self._gather_queries(q_local, q_local_csr)
        d, s = self._local_pair(all_q, all_csr, 2 * k)
        d, s = self._exchange([d, s], 2 * k, nb)
        return self.rrf(d, s, k)

    # ------------------------------------------------------- plugin call (mixed branches)

    def search(self, q_local: torch.Tensor, q_local_csr, mode: str, k: int,
               digest: int = 0) -> TopK:
        """One collective search_batch call of MI355XRetriever (num_gpus > 1). Unlike the
        dense / sparse / hybrid steps above (the bench's lockstep batches), the ranks' calls may
        differ in batch size and branch: the reference's search() is an independent per-call
        operation (retrieval/qdrant.py:227-352, branch chosen per call at 272-332), so a rank
        whose query has no lexical weights (sparse=None: dense) can meet one that searches
        hybrid. A fixed-size header is all-gathered first (batch size, top_k, branch, the
        caller's digest of collection + filter, whether the rank can search sparse); every rank
        reads the same header, so a top_k or filter disagreement raises ValueError on every
        rank alike instead of leaving some ranks waiting in a collective. Then the queries
        (padded to the largest batch; term slots always present when any rank needs them) and
        both candidate lists travel in one all-gather each, and each rank takes its own branch's
        answer: the dense or sparse merged list, or RRF of the two (lists of 2k when any rank
        fuses; the first k of a merged 2k list are the global top k).
        mode: "dense" (or "legacy_dense"), "sparse" or "hybrid"; q_local_csr may be None for
        dense."""
        code = {"dense": 0, "legacy_dense": 0, "sparse": 1, "hybrid": 2}[mode]
        nb = int(q_local.shape[0])
        dev = q_local.device
        hdr = torch.tensor([nb, k, code, int(digest) & ((1 << 62) - 1),
                            int(self.local_sparse is not None)], dtype=torch.int64, device=dev)
        h = self._gather(hdr).cpu()                        # [G, 5], identical on every rank
        if not bool((h[:, 1] == k).all()):
            raise ValueError(f"sharded search: top_k differs across ranks ({h[:, 1].tolist()})")
        if not bool((h[:, 3] == h[0, 3]).all()):
            raise ValueError("sharded search: collection or filter differs across ranks")
        codes = set(h[:, 2].tolist())
        need_sparse = bool(codes & {1, 2})
        if need_sparse and not bool(h[:, 4].all()):
            raise ValueError("sharded search: a rank's collection has no sparse vectors")
        nb_max = int(h[:, 0].max())
        if nb_max == 0:
            return _head(None, 0, k, dev)
        nbs = h[:, 0].tolist()
        self._live = None
        if any(n != nb_max for n in nbs):
            self._live = torch.cat([torch.arange(g * nb_max, g * nb_max + n, dtype=torch.int64)
                                    for g, n in enumerate(nbs)]).to(dev)
        try:
            return self._search_padded(q_local, q_local_csr, code, codes, need_sparse, nb, nb_max,
                                       k, dev)
        finally:
            self._live = None

    def _search_padded(self, q_local, q_local_csr, code: int, codes: set, need_sparse: bool,
                       nb: int, nb_max: int, k: int, dev) -> TopK:
        q_pad = _pad_rows(q_local, nb_max)
        csr = None
        if need_sparse:
            csr = q_local_csr if q_local_csr is not None and code != 0 else _empty_csr(nb, dev)
            csr = _pad_csr_rows(csr, nb_max)
        if codes == {0}:
            out = self.dense(q_pad, k)
        elif codes == {1}:
            out = self.sparse(csr, k)
        elif codes == {2}:
            out = self.hybrid(q_pad, csr, k)
        else:
            kl = 2 * k if 2 in codes else k
            # two or more branches: some rank needs sparse lists and some dense ones
            all_q, all_csr = self._gather_queries(q_pad, csr)
            d, s = self._local_pair(all_q, all_csr, kl)
            d, s = self._exchange([d, s], kl, nb_max)
            out = (_head(d, nb_max, k) if code == 0 else _head(s, nb_max, k) if code == 1
                   else self.rrf(d, s, k))
        return _head(out, nb, k) if nb != nb_max else out

    def _dense_local(self, all_q: torch.Tensor, k: int) -> TopK:
        """The local dense scan of the gathered batch. Inside search() with ranks of different
        batch sizes only the real queries are scanned: a padding row (a copy of the rank's first
        query, or for an empty rank no query at all) has no owner, and an empty rank's padding
        used to be a zero vector, which ties every row at cosine 0, cannot be certified and sent
        every rank through the full-shard collect pass. Padding rows get empty lists."""
        live = self._live
        if live is None:
            self.scanned_queries = int(all_q.shape[0])
            t = self.local_dense(all_q, k)
            self.last_dense_flags = t.flags
            return t
        self.scanned_queries = int(live.numel())
        n = int(all_q.shape[0])
        if live.device != all_q.device:
            live = live.to(all_q.device)
        t = self.local_dense(all_q.index_select(0, live).contiguous(), k)
        self.last_dense_flags = t.flags
        return _scatter_rows(t, live, n, k)

    def _local_pair(self, all_q, all_csr, k: int) -> tuple[TopK, TopK]:
        if not all_q.is_cuda:
            return self._dense_local(all_q, k), self.local_sparse(all_csr, k)
        if self._side is None:
            self._side = torch.cuda.Stream(device=all_q.device)
        main = torch.cuda.current_stream()
        self._side.wait_stream(main)
        for t in all_csr:
            t.record_stream(self._side)
        with torch.cuda.stream(self._side):
            s = self.local_sparse(all_csr, k)
        d = self._dense_local(all_q, k)
        main.wait_stream(self._side)
        for t in s.tensors():
            t.record_stream(main)
        return d, s


def _head(t: TopK | None, n: int, k: int, dev=None) -> TopK:
    """The first n queries and first k entries of a merged list (None: an empty answer)."""
    if t is None:
        return TopK(scores=torch.empty((0, k), dtype=torch.float32, device=dev),
                    ids=torch.empty((0, k), dtype=torch.int64, device=dev),
                    rank=torch.empty((0, k), dtype=torch.float64, device=dev),
                    count=torch.empty(0, dtype=torch.int32, device=dev))
    rank = t.rank
    return TopK(scores=t.scores[:n, :k].contiguous(), ids=t.ids[:n, :k].contiguous(),
                rank=None if rank is None else rank[:n, :k].contiguous(),
                count=t.count[:n].clamp(max=k).to(torch.int32))


def _scatter_rows(t: TopK, rows: torch.Tensor, n: int, k: int) -> TopK:
    """Lists of the selected gathered rows -> lists of all n rows (the others empty: count 0)."""
    dev = t.ids.device
    out = TopK(scores=torch.full((n, k), float("-inf"), dtype=torch.float32, device=dev),
               ids=torch.full((n, k), -1, dtype=torch.int64, device=dev),
               rank=torch.full((n, k), float("-inf"), dtype=torch.float64, device=dev),
               count=torch.zeros(n, dtype=torch.int32, device=dev))
    out.scores.index_copy_(0, rows, t.scores.to(torch.float32))
    out.ids.index_copy_(0, rows, t.ids)
    out.rank.index_copy_(0, rows, t.rank.to(torch.float64))
    out.count.index_copy_(0, rows, t.count.to(torch.int32))
    if t.flags is not None:
        out.flags = torch.zeros(n, dtype=torch.int32, device=dev)
        out.flags.index_copy_(0, rows, t.flags.to(torch.int32))
    return out


def _pad_rows(q: torch.Tensor, n: int) -> torch.Tensor:
    """q [nb, dim] -> [n, dim]: padding rows copy row 0 (zeros for an empty batch). The dense
    scan of search() skips them (ShardedSearch._dense_local); their answers are sliced away."""
    nb = int(q.shape[0])
    if nb == n:
        return q
    fill = q[:1].expand(n - nb, -1) if nb else torch.zeros((n, q.shape[1]), dtype=q.dtype,
                                                                device=q.device)[nb:]
    return torch.cat([q, fill], dim=0).contiguous()


def _empty_csr(n: int, dev) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """n queries without terms (a dense-branch rank's part of a gathered sparse batch); the term
    arrays hold one unused entry so their device pointers are never null."""
    return (torch.zeros(n + 1, dtype=torch.int32, device=dev),
            torch.zeros(1, dtype=torch.int32, device=dev),
            torch.zeros(1, dtype=torch.float32, device=dev))


def _pad_csr_rows(csr, n: int):
    """A query CSR of nb rows -> n rows (the extra rows empty)."""
    indptr, idx, val = csr
    nb = int(indptr.numel()) - 1
    if nb == n:
        return csr
    tail = indptr[-1:].expand(n - nb).to(indptr.dtype)
    return torch.cat([indptr, tail]).contiguous(), idx, val
