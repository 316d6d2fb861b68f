"""The dense second pass (round 3): int8 collect + exact rescore of the queries the first pass
could not certify, the scattered int8 image order, and the int8 first pass up to k = 64 (the
reference's default hybrid prefetch is 40: QueryPipeline.query -> search(top_k=20) -> dense
prefetch limit 2 * 20, src/audio_rag/retrieval/qdrant.py:281-293).

Every answer must be bit-identical to oracle.dense_topk (exact COSINE ranking of the fp16 inputs,
ties by ordinal) on corpora built to defeat the first pass: the clustered / anisotropic corpus of
audio_rag_amd.synthetic (shared mean direction, lecture topics, overlapping-chunk runs of
near-duplicate ordinals, exact re-uploads), a pile of > 4096 identical rows (the collect list
overflows: the second-pass merge scores every row itself), filters, and 65-600-query calls (the
grouped and tiled first passes, several collect blocks).
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _u16(t: torch.Tensor) -> np.ndarray:
    return t.cpu().numpy().view(np.uint16)


def _run(idx, q, k, mask=None):
    out = idx.topk(q, k, row_mask=mask)
    torch.cuda.synchronize()
    return {f: getattr(out, f).cpu().numpy() for f in ("ids", "scores", "rank", "count", "flags")}


def _assert_same(got, ref):
    np.testing.assert_array_equal(got["count"], ref.count)
    for b in range(ref.count.shape[0]):
        c = ref.count[b]
        np.testing.assert_array_equal(got["ids"][b, :c], ref.ids[b, :c], err_msg=f"query {b}")
        np.testing.assert_array_equal(got["rank"][b, :c], ref.rank[b, :c], err_msg=f"query {b}")
        np.testing.assert_array_equal(got["scores"][b, :c], ref.scores[b, :c], err_msg=f"query {b}")


@pytest.fixture(scope="module")
def clustered(gpu):
    from audio_rag_amd.retrieval.device import DenseIndex
    from audio_rag_amd.synthetic import make_clustered_queries, make_clustered_rows

    n = 60000
    rows = make_clustered_rows(0, n, 1024, gpu)
    qs = make_clustered_queries(600, n, 1024, gpu, seed=11)
    return DenseIndex(rows, ordinal_base=3), rows, qs


@pytest.mark.parametrize("k", [5, 20, 40, 64, 100])
def test_clustered_matches_oracle(clustered, oracle_mod, k):
    idx, rows, qs = clustered
    q = qs[:64].contiguous()
    got = _run(idx, q, k)
    _assert_same(got, oracle_mod.dense_topk(_u16(rows), _u16(q), k, ordinal_base=3))
    assert set(np.unique(got["flags"])) <= {1, 2}


@pytest.mark.parametrize("nq", [100, 300, 600])
def test_clustered_multiblock_matches_oracle(clustered, oracle_mod, nq):
    """65-128 queries: grouped int8 first pass; > 128: the tiled fp16 first pass; the uncertified
    queries of the call are dealt to as many collect blocks as they need."""
    idx, rows, qs = clustered
    q = qs[:nq].contiguous()
    for k in (5, 40):
        got = _run(idx, q, k)
        _assert_same(got, oracle_mod.dense_topk(_u16(rows), _u16(q), k, ordinal_base=3))


def test_clustered_with_filter(clustered, oracle_mod):
    idx, rows, qs = clustered
    n = rows.shape[0]
    keep = np.zeros((n + 63) // 64, dtype=np.uint64)
    on = np.random.default_rng(4).random(n) < 0.4
    for r in np.flatnonzero(on):
        keep[r >> 6] |= np.uint64(1) << np.uint64(r & 63)
    mask = torch.from_numpy(keep.view(np.int64)).to(rows.device)
    q = qs[64:128].contiguous()
    for k in (5, 40):
        got = _run(idx, q, k, mask)
        _assert_same(got, oracle_mod.dense_topk(_u16(rows), _u16(q), k, ordinal_base=3,
                                                row_mask=keep))


def test_duplicate_pile_overflows_collect_list(gpu, oracle_mod):
    """5000 identical rows at the top of every query: more rows reach the threshold than the
    collect list holds (4096), so the second-pass merge scores the whole store; ties go by
    ordinal."""
    from audio_rag_amd.retrieval.device import DenseIndex

    base = oracle_mod.unit_fp16(12000, 1024, seed=91)
    v = oracle_mod.unit_fp16(1, 1024, seed=92)
    rows = np.concatenate([base[:3000], np.repeat(v, 5000, axis=0), base[3000:]])
    qs = np.concatenate([v, oracle_mod.unit_fp16(7, 1024, seed=93)])
    idx = DenseIndex(torch.from_numpy(rows.view(np.float16)).to(gpu))
    q = torch.from_numpy(qs.view(np.float16)).to(gpu)
    got = _run(idx, q, 10)
    ref = oracle_mod.dense_topk(rows, qs, 10)
    _assert_same(got, ref)
    assert got["flags"][0] == 2
    assert list(got["ids"][0]) == list(range(3000, 3010))


@pytest.mark.parametrize("k", [1, 40, 240])
def test_overflow_helpers_two_piles_filtered(gpu, oracle_mod, k):
    """Two queries whose lists overflow in one call (two piles of 6500 identical rows, 4333 of them unfiltered), a row
    filter that drops every third pile row, ordinal_base 7, k up to 240: the helper workgroups
    (one 1/n_help slice of the shard each, n_help = min(64, 4096 / k)) find each pile's top-k,
    and the last helper per query merges them; ties go by ordinal."""
    from audio_rag_amd.retrieval.device import DenseIndex

    base = oracle_mod.unit_fp16(9000, 1024, seed=97)
    v1 = oracle_mod.unit_fp16(1, 1024, seed=98)
    v2 = oracle_mod.unit_fp16(1, 1024, seed=99)
    rows = np.concatenate([base[:2000], np.repeat(v1, 6500, axis=0), base[2000:5000],
                           np.repeat(v2, 6500, axis=0), base[5000:]])
    qs = np.concatenate([v1, oracle_mod.unit_fp16(5, 1024, seed=100), v2])
    n = rows.shape[0]
    keep = np.zeros((n + 63) // 64, dtype=np.uint64)
    for r in range(n):
        if not (2000 <= r < 8500 or 11500 <= r < 18000) or r % 3:
            keep[r >> 6] |= np.uint64(1) << np.uint64(r & 63)
    idx = DenseIndex(torch.from_numpy(rows.view(np.float16)).to(gpu), ordinal_base=7)
    q = torch.from_numpy(qs.view(np.float16)).to(gpu)
    mask = torch.from_numpy(keep.view(np.int64)).to(gpu)
    got = _run(idx, q, k, mask)
    ref = oracle_mod.dense_topk(rows, qs, k, ordinal_base=7, row_mask=keep)
    _assert_same(got, ref)
    assert got["flags"][0] == 2 and got["flags"][-1] == 2


def test_fewer_valid_rows_than_k(gpu, oracle_mod):
    """A filter leaving 3 rows: the threshold is -inf and the collect pass returns them all."""
    from audio_rag_amd.retrieval.device import DenseIndex

    rows = oracle_mod.unit_fp16(40000, 1024, seed=95)
    qs = oracle_mod.unit_fp16(16, 1024, seed=96)
    keep = np.zeros((rows.shape[0] + 63) // 64, dtype=np.uint64)
    for r in (5, 17000, 39999):
        keep[r >> 6] |= np.uint64(1) << np.uint64(r & 63)
    idx = DenseIndex(torch.from_numpy(rows.view(np.float16)).to(gpu))
    q = torch.from_numpy(qs.view(np.float16)).to(gpu)
    mask = torch.from_numpy(keep.view(np.int64)).to(gpu)
    got = _run(idx, q, 5, mask)
    _assert_same(got, oracle_mod.dense_topk(rows, qs, 5, row_mask=keep))
    assert (got["count"] == 3).all()


@pytest.mark.parametrize("k", [20, 40, 64])
def test_int8_pass_certifies_large_k_at_100k(gpu, oracle_mod, k):
    """Random unit rows: the int8 first pass with a 256-row rescore certifies k up to 64."""
    from audio_rag_amd import _armi
    from audio_rag_amd.retrieval.device import DenseIndex

    rows = oracle_mod.unit_fp16(100000, 1024, seed=700 + k)
    qs = oracle_mod.unit_fp16(64, 1024, seed=701 + k)
    idx = DenseIndex(torch.from_numpy(rows.view(np.float16)).to(gpu))
    assert idx.scan_form(64, k) == _armi.SCAN_INT8_FILTER
    got = _run(idx, torch.from_numpy(qs.view(np.float16)).to(gpu), k)
    assert (got["flags"] == 1).mean() >= 0.95, got["flags"]
    _assert_same(got, oracle_mod.dense_topk(rows, qs, k))


@pytest.mark.parametrize("n", [1, 31, 33, 1000, 32 * 97 + 5])
def test_scattered_image_odd_sizes(gpu, oracle_mod, n):
    """Image orders of tiny and ragged stores (T = 1, padding inside tiles) keep every row."""
    from audio_rag_amd.retrieval.device import DenseIndex

    rows = oracle_mod.unit_fp16(n, 512, seed=800 + n)
    qs = np.concatenate([rows[: min(n, 8)], oracle_mod.unit_fp16(8, 512, seed=801)])
    idx = DenseIndex(torch.from_numpy(rows.view(np.float16)).to(gpu), ordinal_base=11)
    for k in (1, 5, 40):
        got = _run(idx, torch.from_numpy(qs.view(np.float16)).to(gpu), k)
        _assert_same(got, oracle_mod.dense_topk(rows, qs, k, ordinal_base=11))
