"""Sharded search over a world_size-2 gloo process group on the CPU: the collective plumbing of
audio_rag_amd/retrieval/shards.py (query all-gather, packed candidate all-gather, per-rank
slicing, merge, hybrid RRF) must give every rank exactly the global answer for its queries.
The per-shard search and the merge are CPU stand-ins built on the oracle (this test checks the
exchange, the GPU kernels are checked by the -m gpu tests)."""

import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parent.parent
N, DIM, B, K = 1500, 256, 5, 7


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _topk_t(ids, scores, rank, count):
    from audio_rag_amd.retrieval.device import TopK

    return TopK(scores=torch.from_numpy(np.ascontiguousarray(scores, dtype=np.float32)),
                ids=torch.from_numpy(np.ascontiguousarray(ids, dtype=np.int64)),
                rank=torch.from_numpy(np.ascontiguousarray(rank, dtype=np.float64)),
                count=torch.from_numpy(np.ascontiguousarray(count, dtype=np.int32)))


def cpu_merge(rank, scores, ids, count, k):
    """Merge [S, B, k] lists by (key desc, ordinal asc) — CPU stand-in of armi_topk_merge_shards."""
    s, b, _ = ids.shape
    out_ids = np.full((b, k), -1, np.int64)
    out_sc = np.full((b, k), -np.inf, np.float32)
    out_rk = np.full((b, k), -np.inf, np.float64)
    out_ct = np.zeros(b, np.int32)
    for q in range(b):
        pool = []
        for sh in range(s):
            for j in range(int(count[sh, q])):
                pool.append((-float(rank[sh, q, j]), int(ids[sh, q, j]), float(scores[sh, q, j])))
        pool.sort()
        for j, (nk, oid, sc) in enumerate(pool[:k]):
            out_ids[q, j], out_sc[q, j], out_rk[q, j] = oid, sc, -nk
        out_ct[q] = min(k, len(pool))
    return _topk_t(out_ids, out_sc, out_rk, out_ct)


def _worker(rank, world, port, out_dir):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from audio_rag_amd.retrieval.shards import ShardedSearch, shard_range
    from oracle import oracle as o

    rows = o.unit_fp16(N, DIM, seed=3)
    csr = o.sparse_corpus(N, seed=4)
    lo, hi = shard_range(N, rank, world)
    shard_csr = (csr[0][lo:hi + 1] - csr[0][lo], csr[1][csr[0][lo]:csr[0][hi]], csr[2][csr[0][lo]:csr[0][hi]])

    def local_dense(q, k):
        r = o.dense_topk(rows[lo:hi], q.numpy().view(np.uint16), k, ordinal_base=lo)
        return _topk_t(r.ids, r.scores, r.rank, r.count)

    def local_sparse(qcsr, k):
        qi, qx, qv = (t.numpy() for t in qcsr)
        r = o.sparse_topk(*shard_csr, qi, qx, qv, k, ordinal_base=lo)
        return _topk_t(r.ids, r.scores, r.scores.astype(np.float64), r.count)

    def merge(rank_, scores, ids, count, k):
        return cpu_merge(rank_.numpy(), scores.numpy(), ids.numpy(), count.numpy(), k)

    def rrf(d, s, k):
        b = d.ids.shape[0]
        ids = np.full((b, k), -1, np.int64)
        sc = np.zeros((b, k), np.float64)
        cnt = np.zeros(b, np.int32)
        for q in range(b):
            f = o.rrf([list(d.ids[q, :d.count[q]].tolist()), list(s.ids[q, :s.count[q]].tolist())], k)
            cnt[q] = len(f)
            for j, (p, v) in enumerate(f):
                ids[q, j], sc[q, j] = p, v
        return _topk_t(ids, sc.astype(np.float32), sc, cnt)

    ss = ShardedSearch(local_dense, merge, local_sparse=local_sparse, rrf=rrf)
    q_all = o.unit_fp16(B * world, DIM, seed=5)
    q_mine = torch.from_numpy(q_all[rank * B:(rank + 1) * B].view(np.float16).copy())
    qi, qx, qv = o.sparse_queries(B * world, seed=6)
    a, b = qi[rank * B], qi[(rank + 1) * B]
    q_csr = (torch.from_numpy(qi[rank * B:(rank + 1) * B + 1] - a), torch.from_numpy(qx[a:b]),
             torch.from_numpy(qv[a:b]))
    d = ss.dense(q_mine, K)
    s = ss.sparse(q_csr, K)
    h = ss.hybrid(q_mine, q_csr, K)
    np.savez(Path(out_dir) / f"rank{rank}.npz", d_ids=d.ids.numpy(), d_rank=d.rank.numpy(),
             d_cnt=d.count.numpy(), s_ids=s.ids.numpy(), s_sc=s.scores.numpy(),
             s_cnt=s.count.numpy(), h_ids=h.ids.numpy(), h_sc=h.rank.numpy(), h_cnt=h.count.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharded_search_equals_global(tmp_path, oracle_mod):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    o = oracle_mod
    rows = o.unit_fp16(N, DIM, seed=3)
    csr = o.sparse_corpus(N, seed=4)
    q_all = o.unit_fp16(B * world, DIM, seed=5)
    qcsr = o.sparse_queries(B * world, seed=6)
    gd = o.dense_topk(rows, q_all, K)
    gs = o.sparse_topk(*csr, *qcsr, K)
    gd2 = o.dense_topk(rows, q_all, 2 * K)
    gs2 = o.sparse_topk(*csr, *qcsr, 2 * K)
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        sl = slice(r * B, (r + 1) * B)
        np.testing.assert_array_equal(z["d_ids"], gd.ids[sl])
        np.testing.assert_array_equal(z["d_rank"][z["d_ids"] >= 0], gd.rank[sl][gd.ids[sl] >= 0])
        np.testing.assert_array_equal(z["d_cnt"], gd.count[sl])
        np.testing.assert_array_equal(z["s_cnt"], gs.count[sl])
        for q in range(B):
            c = gs.count[sl][q]
            np.testing.assert_array_equal(z["s_ids"][q, :c], gs.ids[sl][q, :c])
            np.testing.assert_array_equal(z["s_sc"][q, :c], gs.scores[sl][q, :c])
            want = o.rrf([list(gd2.ids[r * B + q, :gd2.count[r * B + q]]),
                          list(gs2.ids[r * B + q, :gs2.count[r * B + q]])], K)
            assert z["h_cnt"][q] == len(want)
            assert [int(x) for x in z["h_ids"][q, :len(want)]] == [p for p, _ in want]
            assert [float(x) for x in z["h_sc"][q, :len(want)]] == [v for _, v in want]


def _mixed_worker(rank, world, port, out_dir):
    """Each rank brings its own batch size and branch to ShardedSearch.search (the plugin's
    collective call): rank 0 / 1 / ... alternate over the cases below."""
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from audio_rag_amd.retrieval.shards import ShardedSearch, shard_range
    from oracle import oracle as o

    rows = o.unit_fp16(N, DIM, seed=3)
    csr = o.sparse_corpus(N, seed=4)
    lo, hi = shard_range(N, rank, world)
    shard_csr = (csr[0][lo:hi + 1] - csr[0][lo], csr[1][csr[0][lo]:csr[0][hi]], csr[2][csr[0][lo]:csr[0][hi]])

    def local_dense(q, k):
        r = o.dense_topk(rows[lo:hi], q.numpy().view(np.uint16), k, ordinal_base=lo)
        return _topk_t(r.ids, r.scores, r.rank, r.count)

    def local_sparse(qcsr, k):
        qi, qx, qv = (t.numpy() for t in qcsr)
        r = o.sparse_topk(*shard_csr, qi, qx, qv, k, ordinal_base=lo)
        return _topk_t(r.ids, r.scores, r.scores.astype(np.float64), r.count)

    def merge(rank_, scores, ids, count, k):
        return cpu_merge(rank_.numpy(), scores.numpy(), ids.numpy(), count.numpy(), k)

    def rrf(d, s, k):
        b = d.ids.shape[0]
        ids = np.full((b, k), -1, np.int64)
        sc = np.zeros((b, k), np.float64)
        cnt = np.zeros(b, np.int32)
        for q in range(b):
            f = o.rrf([list(d.ids[q, :d.count[q]].tolist()), list(s.ids[q, :s.count[q]].tolist())], k)
            cnt[q] = len(f)
            for j, (p, v) in enumerate(f):
                ids[q, j], sc[q, j] = p, v
        return _topk_t(ids, sc.astype(np.float32), sc, cnt)

    ss = ShardedSearch(local_dense, merge, local_sparse=local_sparse, rrf=rrf)
    q_all = o.unit_fp16(B * world, DIM, seed=5)
    qi, qx, qv = o.sparse_queries(B * world, seed=6)
    out = {}
    for case, plan in enumerate(MIXED_CASES):
        mode, nb, empty_terms = plan[rank % len(plan)]
        g0 = rank * B
        q_mine = torch.from_numpy(q_all[g0:g0 + nb].view(np.float16).copy())
        q_csr = None
        if mode != "dense":
            a, b = qi[g0], qi[g0 + nb]
            ip = qi[g0:g0 + nb + 1] - a
            if empty_terms:  # every query an empty SparseVector: hybrid of the dense list alone
                ip = np.zeros_like(ip)
            q_csr = (torch.from_numpy(ip), torch.from_numpy(qx[a:b] if b > a else qx[:1]),
                     torch.from_numpy(qv[a:b] if b > a else qv[:1]))
        t = ss.search(q_mine, q_csr, mode, K, digest=7)
        out[f"c{case}_scanned"] = ss.scanned_queries
        out[f"c{case}_ids"] = t.ids.numpy()
        out[f"c{case}_sc"] = t.rank.numpy()
        out[f"c{case}_cnt"] = t.count.numpy()
    # disagreements raise on every rank (no rank left waiting in a collective)
    for kk, dg in ((K + rank, 7), (K, 7 + rank)):
        try:
            ss.search(torch.from_numpy(q_all[:2].view(np.float16).copy()), None, "dense", kk, dg)
            out["raised"] = out.get("raised", 0)
        except ValueError:
            out["raised"] = out.get("raised", 0) + 1
    t = ss.search(torch.from_numpy(q_all[:2].view(np.float16).copy()), None, "dense", K, 7)
    out["after_ids"] = t.ids.numpy()
    np.savez(Path(out_dir) / f"mixed{rank}.npz", **out)
    dist.barrier()
    dist.destroy_process_group()


# per case: (branch, batch size, empty term lists) of rank 0, rank 1 (ranks cycle over the list)
MIXED_CASES = [
    [("hybrid", B, False), ("dense", B - 2, False)],
    [("sparse", 2, False), ("hybrid", B, True)],
    [("dense", B, False), ("sparse", B - 1, False)],
    [("hybrid", 0, False), ("hybrid", 3, False)],
    [("dense", 0, False), ("hybrid", B, False)],
]


def test_two_rank_mixed_branches_and_sizes(tmp_path, oracle_mod):
    """The plugin's collective call with different branches / batch sizes per rank (a rank whose
    query has sparse=None searches dense while another fuses): every rank gets the global answer
    of its own branch; a top_k or filter disagreement raises on both ranks, and the group stays
    usable afterwards."""
    world = 2
    mp.spawn(_mixed_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    o = oracle_mod
    rows = o.unit_fp16(N, DIM, seed=3)
    csr = o.sparse_corpus(N, seed=4)
    q_all = o.unit_fp16(B * world, DIM, seed=5)
    qi, qx, qv = o.sparse_queries(B * world, seed=6)

    def want(mode, g, empty):
        one = (np.array([0, 0 if empty else qi[g + 1] - qi[g]], np.int32), qx[qi[g]:qi[g + 1]],
               qv[qi[g]:qi[g + 1]])
        if mode == "dense":
            d = o.dense_topk(rows, q_all[g:g + 1], K)
            return list(d.ids[0, :d.count[0]]), list(d.rank[0, :d.count[0]])
        if mode == "sparse":
            s = o.sparse_topk(*csr, *one, K)
            return list(s.ids[0, :s.count[0]]), [float(x) for x in s.scores[0, :s.count[0]]]
        d = o.dense_topk(rows, q_all[g:g + 1], 2 * K)
        s = o.sparse_topk(*csr, *one, 2 * K)
        f = o.rrf([list(d.ids[0, :d.count[0]]), list(s.ids[0, :s.count[0]])], K)
        return [p for p, _ in f], [v for _, v in f]

    for r in range(world):
        z = np.load(tmp_path / f"mixed{r}.npz")
        assert int(z["raised"]) == 2, r
        for case, plan in enumerate(MIXED_CASES):
            # only real queries reach the local dense scan: an empty rank's batch is padding,
            # never scanned (a zero-vector padding query cannot be certified: full collect pass)
            nbs = [plan[g % len(plan)][1] for g in range(world)]
            want_scanned = sum(nbs) if len(set(nbs)) > 1 else world * nbs[0]
            assert int(z[f"c{case}_scanned"]) == want_scanned, (r, case)
        gd = o.dense_topk(rows, q_all[:2], K)
        np.testing.assert_array_equal(z["after_ids"], gd.ids)
        for case, plan in enumerate(MIXED_CASES):
            mode, nb, empty = plan[r % len(plan)]
            assert z[f"c{case}_ids"].shape == (nb, K), (r, case)
            for q in range(nb):
                ids, sc = want(mode, r * B + q, empty)
                c = int(z[f"c{case}_cnt"][q])
                assert c == len(ids), (r, case, q)
                assert [int(x) for x in z[f"c{case}_ids"][q, :c]] == [int(x) for x in ids], (r, case, q)
                assert [float(x) for x in z[f"c{case}_sc"][q, :c]] == [float(x) for x in sc], (r, case, q)


def test_pad_unpad_csr_roundtrip():
    """The fixed-slot query layout of the one-collective query exchange: ragged, empty and
    full (MAX_QUERY_TERMS) queries survive pad -> unpad with the CSR order intact."""
    from audio_rag_amd.retrieval.shards import MAX_QUERY_TERMS, pack_rows, pad_csr, unpack_rows, unpad_csr

    rng = np.random.default_rng(0)
    lens = [0, 3, MAX_QUERY_TERMS, 1, 0, 17]
    indptr = np.zeros(len(lens) + 1, np.int32)
    indptr[1:] = np.cumsum(lens)
    idx = rng.integers(0, 250002, indptr[-1]).astype(np.int32)
    val = rng.random(indptr[-1]).astype(np.float32)
    t = lambda a: torch.from_numpy(a)
    cnt, pi, pv = pad_csr(t(indptr), t(idx), t(val))
    assert cnt.tolist() == lens and pi.shape == (len(lens), MAX_QUERY_TERMS)
    dense = torch.randn(len(lens), 8, dtype=torch.float64)
    buf, layout = pack_rows([dense, cnt, pi, pv])
    d2, c2, i2, v2 = unpack_rows(buf, layout)
    assert torch.equal(d2, dense)
    ip2, ix2, vx2 = unpad_csr(c2, i2, v2)
    assert ip2.tolist() == indptr.tolist()
    n = int(indptr[-1])
    assert ix2[:n].tolist() == idx.tolist() and vx2[:n].tolist() == val.tolist()


def test_unpack_single_row_of_mixed_dtypes():
    """One query's row of a packed hybrid exchange (bench.py's single-query probe at WORLD_SIZE 1:
    the slice is contiguous, so unpack_rows views it in place) with 8-byte parts after 4-byte
    ones in the caller's order: every part must come back intact (a float64 part at byte offset
    204 could not be viewed before the element-size ordering)."""
    from audio_rag_amd.retrieval.shards import pack_rows, unpack_rows

    k = 10
    parts = [torch.randn(3, k, dtype=torch.float64), torch.arange(3 * k).reshape(3, k),
             torch.randn(3, k), torch.arange(3, dtype=torch.int32).view(3, 1),
             torch.randn(3, k, dtype=torch.float64), torch.arange(3 * k).reshape(3, k) + 7,
             torch.randn(3, k), torch.arange(3, dtype=torch.int32).view(3, 1) + 1]
    buf, layout = pack_rows(parts)
    g = buf.reshape(1, 3, -1)
    for r in range(3):
        got = unpack_rows(g[:, r:r + 1], layout)
        for a, b in zip(got, parts):
            assert a.dtype == b.dtype and torch.equal(a.reshape(b[r:r + 1].shape), b[r:r + 1])


def test_pad_csr_ignores_trailing_entries():
    """A CSR whose index / value arrays run past indptr[-1] (bench.py's single-query probe keeps
    the whole batch's term arrays under a one-query indptr) pads only the live entries; the
    trailing ones must not be written anywhere (they went past the buffer before: a GPU fault in
    the N > 1 hybrid rehearsal)."""
    from audio_rag_amd.retrieval.shards import pad_csr, unpad_csr

    indptr = torch.tensor([0, 3], dtype=torch.int32)
    idx = torch.arange(10, 10 + 700, dtype=torch.int32)  # 700 entries, 3 live
    val = torch.arange(700, dtype=torch.float32)
    cnt, pi, pv = pad_csr(indptr, idx, val)
    assert cnt.tolist() == [3] and pi[0, :3].tolist() == [10, 11, 12] and pi[0, 3:].eq(0).all()
    ip2, ix2, vx2 = unpad_csr(cnt, pi, pv)
    assert ip2.tolist() == [0, 3] and ix2[:3].tolist() == [10, 11, 12] and vx2[:3].tolist() == [0, 1, 2]
    empty = pad_csr(torch.zeros(1, dtype=torch.int32), idx, val)
    assert empty[1].shape == (0, 256)
