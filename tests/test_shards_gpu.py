"""Sharded search with the real kernels: G ranks (one process each) share cuda:0 and exchange over
gloo (RCCL refuses two ranks on one device), so ShardedSearch (audio_rag_amd/retrieval/shards.py)
runs exactly what bench.py runs at N = G — the query all-gather, the local libarmi scans of all
G*B queries (grouped int8 scan at 128 queries, four-wave tiled scan at 256), the packed candidate
all-gather, armi_topk_merge_shards and RRF after the merge — and every rank must hold the global
answer of the oracle over the whole corpus for its own queries. The collective backend is the
only difference from an N-GPU run. Reference: a single Qdrant collection answers the same
search (retrieval/qdrant.py:281-332)."""

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
N, DIM, B, K = 24000, 1024, 64, 5
VOCAB = 250002


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir, packed):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from audio_rag_amd.retrieval.device import (DenseIndex, SparseIndex, merge_shards,
                                                merge_shards_packed, rrf_fuse)
    from audio_rag_amd.retrieval.shards import ShardedSearch, shard_range
    from oracle import oracle as o

    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    rows = o.unit_fp16(N, DIM, seed=3)
    indptr, indices, values = o.sparse_corpus(N, seed=4)
    lo, hi = shard_range(N, rank, world)
    dense = DenseIndex(t(rows[lo:hi].view(np.float16)), ordinal_base=lo)
    a, b = indptr[lo], indptr[hi]
    sparse = SparseIndex(t(indptr[lo:hi + 1] - a), t(indices[a:b]), t(values[a:b]), VOCAB, lo)
    ws = torch.empty(dense.workspace_bytes(world * B, 2 * K), dtype=torch.uint8, device=dev)
    sws = torch.empty(sparse.workspace_bytes(world * B, 2 * K), dtype=torch.uint8, device=dev)
    ss = ShardedSearch(lambda q, kk: dense.topk(q, kk, workspace=ws), merge_shards,
                       local_sparse=lambda c, kk: sparse.topk(*c, kk, workspace=sws),
                       rrf=lambda x, y, kk: rrf_fuse(x, y, kk),
                       merge_packed=merge_shards_packed if packed else None)
    q_all = o.unit_fp16(B * world, DIM, seed=5)
    q_mine = t(q_all[rank * B:(rank + 1) * B].view(np.float16))
    qi, qx, qv = o.sparse_queries(B * world, seed=6)
    qa, qb = qi[rank * B], qi[(rank + 1) * B]
    q_csr = (t(qi[rank * B:(rank + 1) * B + 1] - qa), t(qx[qa:qb]), t(qv[qa:qb]))
    d = ss.dense(q_mine, K)
    s = ss.sparse(q_csr, K)
    h = ss.hybrid(q_mine, q_csr, K)
    torch.cuda.synchronize()
    c = lambda x: x.cpu().numpy()
    np.savez(Path(out_dir) / f"rank{rank}.npz", d_ids=c(d.ids), d_rank=c(d.rank), d_cnt=c(d.count),
             s_ids=c(s.ids), s_sc=c(s.scores), s_cnt=c(s.count), h_ids=c(h.ids), h_sc=c(h.rank),
             h_cnt=c(h.count))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world,packed", [(2, True), (4, True), (2, False)])
def test_sharded_search_real_kernels_equal_global(tmp_path, oracle_mod, world, packed):
    """packed: the merge reads the gathered exchange rows in place (armi_topk_merge_shards_packed,
    what bench.py runs); otherwise unpacked per-field copies into armi_topk_merge_shards."""
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), packed), nprocs=world, join=True)
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
        np.testing.assert_array_equal(z["d_rank"], gd.rank[sl])
        np.testing.assert_array_equal(z["d_cnt"], gd.count[sl])
        np.testing.assert_array_equal(z["s_cnt"], gs.count[sl])
        for q in range(B):
            c = gs.count[sl][q]
            np.testing.assert_array_equal(z["s_ids"][q, :c], gs.ids[sl][q, :c])
            np.testing.assert_array_equal(z["s_sc"][q, :c], gs.scores[sl][q, :c])
            g = r * B + q
            want = o.rrf([list(gd2.ids[g, :gd2.count[g]]), list(gs2.ids[g, :gs2.count[g]])], K)
            assert z["h_cnt"][q] == len(want)
            assert [int(x) for x in z["h_ids"][q, :len(want)]] == [p for p, _ in want]
            assert [float(x) for x in z["h_sc"][q, :len(want)]] == [v for _, v in want]


@pytest.mark.gpu
def test_query_slots_pack_unpack_match_host(gpu):
    """armi_query_slots_pack / _unpack (the sharded hybrid step's query exchange on the GPU)
    against the host torch form of the same exchange: ragged, empty, full (MAX_QUERY_TERMS) and
    over-long (truncated) queries, trailing CSR entries past indptr[-1], 1,300 queries (the
    unpack's prefix sum runs over two 1,024-query rounds)."""
    from audio_rag_amd.retrieval.shards import (MAX_QUERY_TERMS, pack_rows, pad_csr, unpack_rows,
                                                unpad_csr)

    rng = np.random.default_rng(5)
    lens = rng.integers(0, 40, 1300)
    lens[[0, 7, 8]] = 0
    lens[3] = MAX_QUERY_TERMS
    lens[5] = MAX_QUERY_TERMS + 9  # truncated by both forms
    indptr = np.zeros(len(lens) + 1, np.int32)
    indptr[1:] = np.cumsum(lens)
    idx = rng.integers(0, 250002, indptr[-1] + 50).astype(np.int32)  # 50 trailing entries
    val = rng.random(indptr[-1] + 50).astype(np.float32)
    host = pad_csr(*(torch.from_numpy(a) for a in (indptr, idx, val)))
    dev = pad_csr(*(torch.from_numpy(a).to(gpu) for a in (indptr, idx, val)))
    for h, d in zip(host, dev):
        assert torch.equal(h, d.cpu())
    # unpack from a packed, gathered-shaped buffer with a leading dense part (odd byte width)
    dense = torch.randint(0, 255, (len(lens), 6), dtype=torch.uint8)
    buf, layout = pack_rows([dense.to(gpu), *dev])
    from audio_rag_amd._armi import call, ptr, stream_handle
    n = len(lens)
    ip = torch.empty(n + 1, dtype=torch.int32, device=gpu)
    ix = torch.empty(n * MAX_QUERY_TERMS, dtype=torch.int32, device=gpu)
    vx = torch.empty(n * MAX_QUERY_TERMS, dtype=torch.float32, device=gpu)
    lc, li, lv = layout[1:]
    call("armi_query_slots_unpack", buf.data_ptr(), int(buf.stride(0)), lc[0], li[0], lv[0], n,
         MAX_QUERY_TERMS, ptr(ip), ptr(ix), ptr(vx), stream_handle())
    want = unpad_csr(*unpack_rows(buf.cpu(), layout)[1:])
    m = int(want[0][-1])
    assert torch.equal(ip.cpu(), want[0])
    assert torch.equal(ix.cpu()[:m], want[1][:m]) and torch.equal(vx.cpu()[:m], want[2][:m])
