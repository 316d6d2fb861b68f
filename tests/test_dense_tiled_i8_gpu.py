"""The int8 x int8 tiled scan (ARMI_SCAN_TILED_INT8: > 128 queries, k <= 5, shards of >= 200k
rows): dense_gemm_scan_w4_kernel<dim, 0, true> over the index's int8 image and the call's int8
queries, keys = certified upper bounds, exact fp16 rescore and certificate in dense_merge_kernel,
collect pass for whatever is not certified. Results must equal the exhaustive exact scan bit for
bit (ids, fp64 ranks, fp32 scores) for every query, with and without a row filter, on an odd row
count (a padded tail image tile, ranges that end inside a 32-row tile) and an ordinal base; a
sample equals the CPU oracle. Reference: Qdrant COSINE search (retrieval/qdrant.py:284-288)."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N, DIM, B = 600_011, 1024, 300
SAMPLE = [0, 1, 127, 128, 255, 256, 299]


@pytest.fixture(scope="module")
def shard(gpu):
    from audio_rag_amd.retrieval.device import DenseIndex
    from audio_rag_amd.synthetic import make_queries, make_rows

    rows = make_rows(0, N, DIM, gpu, seed=7)
    idx = DenseIndex(rows, ordinal_base=1_000_000)
    q = make_queries(1, B, DIM, gpu, seed=8)[0].contiguous()
    torch.cuda.synchronize()
    yield dict(idx=idx, rows=rows, q=q)
    idx.close()
    torch.cuda.empty_cache()


def _same(a, b):
    for f in ("count", "ids", "rank", "scores"):
        np.testing.assert_array_equal(getattr(a, f).cpu().numpy(), getattr(b, f).cpu().numpy(),
                                      err_msg=f)


@pytest.mark.parametrize("k", [1, 5])
def test_tiled_i8_equals_exact_and_oracle(shard, oracle_mod, k):
    from audio_rag_amd import _armi

    idx, q = shard["idx"], shard["q"]
    assert idx.scan_form(B, k) == _armi.SCAN_TILED_INT8
    fast = idx.topk(q, k)
    exact = idx.topk(q, k, exact=True)
    torch.cuda.synchronize()
    cert = fast.flags.eq(1).float().mean().item()
    print(f"tiled int8 scan {N} x {B}, k={k}: certified fraction {cert:.4f}")
    assert cert >= 0.95  # the fast path answers (nearly) every query itself
    _same(fast, exact)
    rows_u16 = shard["rows"].cpu().numpy().view(np.uint16)
    qs = q.cpu().numpy().view(np.uint16)[SAMPLE]
    want = oracle_mod.dense_topk(rows_u16, qs, k, ordinal_base=1_000_000)
    np.testing.assert_array_equal(fast.ids.cpu().numpy()[SAMPLE], want.ids)
    np.testing.assert_array_equal(fast.scores.cpu().numpy()[SAMPLE], want.scores)


def test_tiled_i8_row_filter(shard):
    """A 40 % row filter, with two all-zero queries in the batch (every enabled row ties at 0:
    the answer is the first enabled ordinals, and no filtered row may slip in)."""
    idx = shard["idx"]
    q = shard["q"].clone()
    q[5] = 0
    q[200] = 0
    g = torch.Generator(device=q.device).manual_seed(3)
    bits = torch.rand(N, generator=g, device=q.device) < 0.4
    words = torch.zeros((N + 63) // 64 * 64, dtype=torch.bool, device=q.device)
    words[:N] = bits
    w = words.view(-1, 64).to(torch.int64)
    mask = (w << torch.arange(64, device=q.device, dtype=torch.int64)).sum(dim=1)
    fast = idx.topk(q, 5, row_mask=mask)
    exact = idx.topk(q, 5, row_mask=mask, exact=True)
    torch.cuda.synchronize()
    _same(fast, exact)
    # every returned row is enabled
    ids = fast.ids.cpu().numpy() - 1_000_000
    assert bits.cpu().numpy()[ids[ids >= 0]].all()
