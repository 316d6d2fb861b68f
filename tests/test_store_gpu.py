"""On-disk chunk store on the GPU: a collection saved and loaded by another retriever answers
every search identically (ids, scores, order), and the per-rank shards opened from the store
merge to the global answer (bit-exact against the CPU oracle)."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_saved_store_searches_identically(gpu, oracle_mod, tmp_path):
    from audio_rag_amd.config import RetrievalConfig
    from audio_rag_amd.retrieval.mi355x import MI355XRetriever

    n = 3000
    rows = oracle_mod.unit_fp16(n, 1024, seed=41).view(np.float16)
    csr = oracle_mod.sparse_corpus(n, seed=42)
    sparse = [(csr[1][csr[0][i]:csr[0][i + 1]], csr[2][csr[0][i]:csr[0][i + 1]]) for i in range(n)]
    payloads = [{"text": f"c{i}", "start": i, "end": i + 1, "speaker": None,
                 "metadata": {"lecture": i % 5}} for i in range(n)]
    a = MI355XRetriever(RetrievalConfig(), 1024)
    a.add_arrays(rows, payloads, sparse=sparse, collection_name="c")
    a.save_collection(tmp_path / "c", "c")
    b = MI355XRetriever(RetrievalConfig(), 1024)
    b.load_collection(tmp_path / "c")
    qi, qx, qv = oracle_mod.sparse_queries(16, seed=43)
    q = oracle_mod.unit_fp16(16, 1024, seed=44).view(np.float16)
    from audio_rag_amd.retrieval.mi355x import QueryBatch

    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(gpu)
    batch = QueryBatch(dense=t(q), sparse_indptr=t(qi), sparse_indices=t(qx), sparse_values=t(qv))
    for st in ("dense", "sparse", "hybrid"):
        for flt in (None, {"lecture": 2}):
            ra, ma = a.search_batch(batch, 10, "c", flt, st)
            rb, mb = b.search_batch(batch, 10, "c", flt, st)
            torch.cuda.synchronize()
            assert ma == mb == st
            assert torch.equal(ra.count.cpu(), rb.count.cpu())
            assert torch.equal(ra.ids.cpu(), rb.ids.cpu())
            assert torch.equal(ra.scores.cpu(), rb.scores.cpu())


def test_store_shards_merge_to_global(gpu, oracle_mod, tmp_path):
    from audio_rag_amd.retrieval.device import merge_shards
    from audio_rag_amd.retrieval.store import open_shard, save_arrays

    n, k = 5001, 7
    rows = oracle_mod.unit_fp16(n, 1024, seed=45)
    save_arrays(tmp_path / "s", "s", rows.view(np.float16), None,
                [{"text": str(i)} for i in range(n)], hybrid=False)
    qs = oracle_mod.unit_fp16(9, 1024, seed=46)
    q = torch.from_numpy(qs.view(np.float16)).to(gpu)
    parts = []
    for r in range(3):
        dense, sparse, sh = open_shard(tmp_path / "s", r, 3, gpu)
        assert sparse is None and dense.ordinal_base == sh.lo
        parts.append(dense.topk(q, k))
    st = lambda f: torch.stack([getattr(p, f) for p in parts])
    m = merge_shards(st("rank"), st("scores"), st("ids"), st("count"), k)
    torch.cuda.synchronize()
    ref = oracle_mod.dense_topk(rows, qs, k)
    np.testing.assert_array_equal(m.ids.cpu().numpy(), ref.ids)
    np.testing.assert_array_equal(m.rank.cpu().numpy(), ref.rank)
