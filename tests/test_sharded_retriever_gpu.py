"""The sharded plugin surface: MI355XRetriever with RetrievalConfig(num_gpus=G), G processes (one
per rank) sharing cuda:0 over gloo (RCCL refuses two ranks on one device; an N-GPU run differs
only in the backend). Every rank add()s the same chunks and keeps its ordinal shard on the device;
search_batch / search are collective calls that return the GLOBAL top-k of each rank's own
queries (dense, sparse-only, hybrid, with a payload filter), and each rank reranks its own query
slice locally with BGEReranker: the answers must equal the oracle's over the whole corpus and the
rerank scores transformers' fp32 cross-encoder within 1e-3.
Reference: one QdrantRetriever over one collection (retrieval/qdrant.py:227-352) and
BGEReranker.rerank (reranking/bge.py:86-147), as AudioRAG wires them (pipeline/orchestrator.py:
48-57, pipeline/query.py:152-198)."""

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
N, DIM, B, K = 6000, 1024, 8, 6
RR_ARCH = dict(num_hidden_layers=2)  # a 2-layer bge-reranker-base: the rerank is rank-local


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _payloads():
    return [{"text": f"chunk {r} lecture {r % 3} words{r % 17}", "start": float(r),
             "end": float(r) + 1.0, "speaker": None, "metadata": {"lecture": r % 3}}
            for r in range(N)]


def _worker(rank, world, port, out_dir):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from audio_rag_amd.config import RetrievalConfig
    from audio_rag_amd.config.schema import RerankingConfig
    from audio_rag_amd.core import EmbeddingResult, SparseVector
    from audio_rag_amd.reranking.bge import BGEReranker
    from audio_rag_amd.retrieval.mi355x import MI355XRetriever
    from oracle import oracle as o

    rows = o.unit_fp16(N, DIM, seed=31)
    ip, ix, iv = o.sparse_corpus(N, seed=32)
    sparse = [(ix[ip[r]:ip[r + 1]], iv[ip[r]:ip[r + 1]]) for r in range(N)]
    cfg = RetrievalConfig(top_k=K, num_gpus=world)
    ret = MI355XRetriever(cfg, DIM)
    ret.add_arrays(rows.view(np.float16), _payloads(), sparse=sparse)
    coll = ret.collection()
    lo, hi = coll.shard_bounds()
    assert coll.dense_index.n_rows == hi - lo and coll.dense_index.ordinal_base == lo
    qd = o.unit_fp16(B * world, DIM, seed=33)
    qi, qx, qv = o.sparse_queries(B * world, seed=34)
    mine = range(rank * B, (rank + 1) * B)
    qf = qd.view(np.float16).astype(np.float32)
    embs = [EmbeddingResult(dense=qf[i].tolist(),
                            sparse=SparseVector(qx[qi[i]:qi[i + 1]].tolist(),
                                                qv[qi[i]:qi[i + 1]].tolist())) for i in mine]
    batch = ret.to_query_batch(embs)
    dense_only = ret.to_query_batch([EmbeddingResult(dense=e.dense) for e in embs])
    out = {}
    for st, qb, flt in (("hybrid", batch, None), ("sparse", batch, None), ("dense", dense_only, None),
                        ("hybrid", batch, {"lecture": 1}), ("dense", dense_only, {"lecture": 2})):
        tk, mode = ret.search_batch(qb, K, None, flt, st)
        res = ret.materialize_batch(tk, mode, coll.name)
        key = f"{st}_{'f' if flt else 'n'}"
        out[key + "_ids"] = np.array([[int(r.chunk.text.split()[1]) for r in rs] + [-1] * (K - len(rs))
                                      for rs in res])
        out[key + "_sc"] = np.array([[r.score for r in rs] + [0.0] * (K - len(rs)) for rs in res])
    # mixed branches and batch sizes across ranks in one collective call (qdrant.py:272-332
    # chooses the branch per call): even ranks fuse / search sparse, odd ranks bring queries
    # without lexical weights (dense) or with empty SparseVectors (hybrid of the dense list alone)
    empty = ret.to_query_batch([EmbeddingResult(dense=e.dense, sparse=SparseVector([], []))
                                for e in embs[:2]])
    for name, (st, qb) in (("mixA", ("hybrid", batch) if rank % 2 == 0 else
                            ("hybrid", ret.to_query_batch([EmbeddingResult(dense=e.dense)
                                                            for e in embs[:B - 3]]))),
                           ("mixB", ("sparse", batch) if rank % 2 == 0 else ("hybrid", empty))):
        tk, mode = ret.search_batch(qb, K, None, None, st)
        out[name + "_mode"] = np.array(mode)
        res = ret.materialize_batch(tk, mode, coll.name)
        out[name + "_ids"] = [[int(r.chunk.text.split()[1]) for r in rs] for rs in res]
        out[name + "_sc"] = [[r.score for r in rs] for rs in res]
        out[name + "_ids"] = np.array([x + [-1] * (K - len(x)) for x in out[name + "_ids"]])
        out[name + "_sc"] = np.array([x + [0.0] * (K - len(x)) for x in out[name + "_sc"]])
    # an empty rank (no queries this call) beside ranks that search hybrid: its padding rows are
    # never scanned, so every scanned dense query is certified (a zero-vector padding query
    # used to tie every row and send each rank through the full-shard collect pass)
    qb = batch if rank % 2 else type(batch)(dense=batch.dense[:0], sparse_indptr=batch.sparse_indptr[:1],
                                           sparse_indices=batch.sparse_indices,
                                           sparse_values=batch.sparse_values)
    tk, mode = ret.search_batch(qb, K, None, None, "hybrid")
    res = ret.materialize_batch(tk, mode, coll.name)
    out["mixC_n"] = np.array(len(res))
    out["mixC_ids"] = np.array([[int(r.chunk.text.split()[1]) for r in rs] + [-1] * (K - len(rs))
                                for rs in res]).reshape(len(res), K)
    out["mixC_sc"] = np.array([[r.score for r in rs] + [0.0] * (K - len(rs))
                               for rs in res]).reshape(len(res), K)
    sh = ret.last_sharded
    out["mixC_scanned"] = np.array(sh.scanned_queries)
    fl = sh.last_dense_flags.cpu().numpy()
    out["mixC_certified"] = np.array(int(np.all((fl & 1) == 1) and np.all((fl & 2) == 0)))
    # a top_k disagreement raises RetrievalError on every rank instead of hanging
    from audio_rag_amd.core.exceptions import RetrievalError

    try:
        ret.search_batch(dense_only, K + rank, None, None, "dense")
        out["raised"] = np.array(0)
    except RetrievalError:
        out["raised"] = np.array(1)
    # search() one query per rank (collective), then the rank-local rerank of its own slice
    rr = BGEReranker(RerankingConfig(top_k=3), device=torch.device("cuda", 0), arch=RR_ARCH)
    rr.load()
    hits = ret.search(embs[0], top_k=K, search_type="hybrid")
    out["single_ids"] = np.array([int(r.chunk.text.split()[1]) for r in hits])
    reranked = rr.rerank(f"query {rank}", hits)
    out["rr_ids"] = np.array([int(r.chunk.text.split()[1]) for r in reranked])
    out["rr_sc"] = np.array([r.score for r in reranked])
    np.savez(Path(out_dir) / f"rank{rank}.npz", **out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_sharded_retriever_plugin_equals_global(tmp_path, oracle_mod, world):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    o = oracle_mod
    from audio_rag_amd.reranking.xlmr import build_reranker
    from audio_rag_amd.text import HashTokenizer, pad_batch, pair_ids

    rows = o.unit_fp16(N, DIM, seed=31)
    csr = o.sparse_corpus(N, seed=32)
    qd = o.unit_fp16(B * world, DIM, seed=33)
    qcsr = o.sparse_queries(B * world, seed=34)
    lect = np.arange(N) % 3

    def mask_of(flt):
        if flt is None:
            return None
        m = np.zeros((N + 63) // 64, dtype=np.uint64)
        for r in np.nonzero(lect == flt)[0]:
            m[r >> 6] |= np.uint64(1) << np.uint64(r & 63)
        return m

    def want(st, flt, g):
        m = mask_of(flt)
        q1 = qd[g:g + 1]
        s_ptr = np.array([0, qcsr[0][g + 1] - qcsr[0][g]], dtype=np.int32)
        s_idx, s_val = qcsr[1][qcsr[0][g]:qcsr[0][g + 1]], qcsr[2][qcsr[0][g]:qcsr[0][g + 1]]
        if st == "dense":
            d = o.dense_topk(rows, q1, K, row_mask=m)
            return list(d.ids[0, :d.count[0]]), list(d.scores[0, :d.count[0]])
        if st == "sparse":
            s = o.sparse_topk(*csr, s_ptr, s_idx, s_val, K, row_mask=m)
            return list(s.ids[0, :s.count[0]]), list(s.scores[0, :s.count[0]])
        d = o.dense_topk(rows, q1, 2 * K, row_mask=m)
        s = o.sparse_topk(*csr, s_ptr, s_idx, s_val, 2 * K, row_mask=m)
        f = o.rrf([list(d.ids[0, :d.count[0]]), list(s.ids[0, :s.count[0]])], K)
        return [p for p, _ in f], [v for _, v in f]

    hf = build_reranker(5, dict(RR_ARCH, attn_implementation="eager"))
    tok = HashTokenizer()
    texts = {r["text"].split()[1]: r["text"] for r in _payloads()}
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        for st, flt in (("hybrid", None), ("sparse", None), ("dense", None), ("hybrid", 1),
                        ("dense", 2)):
            key = f"{st}_{'f' if flt is not None else 'n'}"
            for q in range(B):
                ids, sc = want(st, flt, r * B + q)
                assert list(z[key + "_ids"][q, :len(ids)]) == [int(x) for x in ids], (r, key, q)
                assert [float(x) for x in z[key + "_sc"][q, :len(sc)]] == [float(x) for x in sc]
        assert int(z["raised"]) == 1, r
        for name in ("mixA", "mixB"):
            mode = str(z[name + "_mode"])
            nq = z[name + "_ids"].shape[0]
            want_mode = {("mixA", 0): "hybrid", ("mixA", 1): "dense", ("mixB", 0): "sparse",
                         ("mixB", 1): "hybrid"}[(name, r % 2)]
            assert mode == want_mode and nq == {("mixA", 1): B - 3, ("mixB", 1): 2}.get((name, r % 2), B)
            for q in range(nq):
                if name == "mixB" and r % 2:  # empty SparseVector: RRF of the dense 2k list alone
                    d = o.dense_topk(rows, qd[r * B + q:r * B + q + 1], 2 * K)
                    f = o.rrf([list(d.ids[0, :d.count[0]]), []], K)
                    ids, sc = [p for p, _ in f], [v for _, v in f]
                else:
                    ids, sc = want(mode, None, r * B + q)
                assert list(z[name + "_ids"][q, :len(ids)]) == [int(x) for x in ids], (r, name, q)
                assert [float(x) for x in z[name + "_sc"][q, :len(sc)]] == [float(x) for x in sc]
        assert int(z["mixC_scanned"]) == B * (world // 2) and int(z["mixC_certified"]) == 1, r
        assert int(z["mixC_n"]) == (B if r % 2 else 0), r
        for q in range(int(z["mixC_n"])):
            ids, sc = want("hybrid", None, r * B + q)
            assert list(z["mixC_ids"][q, :len(ids)]) == [int(x) for x in ids], (r, "mixC", q)
            assert [float(x) for x in z["mixC_sc"][q, :len(sc)]] == [float(x) for x in sc]
        ids, _ = want("hybrid", None, r * B)
        assert list(z["single_ids"]) == [int(x) for x in ids]
        # rank-local rerank of its own slice vs transformers fp32 (bge.py:119-123)
        qt = tok.tokenize(f"query {r}")
        pairs = [pair_ids(qt, tok.tokenize(texts[str(i)]), 512) for i in ids]
        pid, pm = pad_batch(pairs)
        with torch.no_grad():
            ref = torch.sigmoid(hf(input_ids=torch.tensor(pid), attention_mask=torch.tensor(pm))
                                .logits[:, 0]).numpy()
        order = np.argsort(-ref, kind="stable")[:3]
        assert list(z["rr_ids"]) == [int(ids[i]) for i in order], r
        np.testing.assert_allclose(z["rr_sc"], ref[order], rtol=0, atol=1e-3)
