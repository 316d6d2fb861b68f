"""HybridGraph (retrieval/device.py): the captured hybrid step (dense top-k, sparse top-k, RRF;
qdrant.py:281-298) replayed over different batches equals the eager ConcurrentHybrid step
exactly (ids, fp64 RRF scores, counts)."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_hybrid_graph_matches_eager(gpu):
    from audio_rag_amd import synthetic
    from audio_rag_amd.retrieval.device import ConcurrentHybrid, DenseIndex, HybridGraph, SparseIndex

    n, batch, pre_k, limit = 30000, 64, 40, 20
    rows = synthetic.make_rows(0, n, 1024, gpu)
    dense = DenseIndex(rows)
    sparse = SparseIndex(*synthetic.make_sparse_rows(0, n, gpu), vocab=synthetic.VOCAB)
    hg = HybridGraph(dense, sparse, batch, pre_k, limit)
    eager = ConcurrentHybrid(gpu)
    for seed in (11, 12, 13):
        g = torch.Generator(device=gpu).manual_seed(seed)
        q = torch.randn((batch, rows.shape[1]), generator=g, device=gpu).half()
        qs = synthetic.make_sparse_queries(batch, gpu, seed)
        want = eager(lambda: dense.topk(q, pre_k), lambda: sparse.topk(*qs, pre_k), qs, limit)
        for got in (hg(q, *qs), hg(hg.pack(q, *qs))):  # per-array copies; one packed copy
            torch.cuda.synchronize()
            assert torch.equal(got.count, want.count)
            assert torch.equal(got.ids, want.ids)
            assert torch.equal(got.rank, want.rank)
    with pytest.raises(ValueError):
        hg(q[:8], *synthetic.make_sparse_queries(8, gpu, 1))
