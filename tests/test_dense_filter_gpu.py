"""The int8 filter pass of the 64-query dense scan (dense_scan_i8_kernel, include/armi.h
armi_dense_scan_form) against the CPU oracle.

The filter ranks rows by an upper bound of their fp16 cosine (int8 image + Cauchy-Schwarz bound of
the quantisation error) and the merge rescores the best bounds exactly, so the answer must stay
bit-identical to oracle.dense_topk (QdrantRetriever.search's dense COSINE ranking,
src/audio_rag/retrieval/qdrant.py:284-288, 316-332) on inputs built to stress the bound: rows
whose components span a wide dynamic range (a few large components, the rest tiny: a large
quantisation error), near-duplicate rows (ties broken by ordinal), zero rows (key 0), and a row
filter.
The int8 first pass serves k <= 64 (fp16 scan beyond), and at 100k random unit rows every query
must be certified (no second pass).
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev(a, gpu):
    return torch.from_numpy(np.ascontiguousarray(a)).to(gpu)


def _index(rows_u16, gpu, base=0):
    from audio_rag_amd.retrieval.device import DenseIndex

    return DenseIndex(_dev(rows_u16.view(np.float16), gpu), ordinal_base=base)


def _run(idx, q_u16, k, gpu, mask=None):
    q = _dev(q_u16.view(np.float16), gpu)
    m = None if mask is None else _dev(mask.view(np.int64), gpu)
    out = idx.topk(q, k, row_mask=m)
    torch.cuda.synchronize()
    return {f: getattr(out, f).cpu().numpy() for f in ("ids", "scores", "rank", "count", "flags")}


def _assert_same(got, ref):
    np.testing.assert_array_equal(got["count"], ref.count)
    for b in range(ref.count.shape[0]):
        c = ref.count[b]
        np.testing.assert_array_equal(got["ids"][b, :c], ref.ids[b, :c], err_msg=f"query {b}")
        np.testing.assert_array_equal(got["rank"][b, :c], ref.rank[b, :c], err_msg=f"query {b}")
        np.testing.assert_array_equal(got["scores"][b, :c], ref.scores[b, :c], err_msg=f"query {b}")


def _to_u16(x: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(x.astype(np.float16)).view(np.uint16)


def _spiky_rows(n: int, dim: int, seed: int) -> np.ndarray:
    """Unit rows with 1-4 large components and the rest ~1e-3: the int8 image keeps the spikes
    and rounds most other components to 0, so the per-row error bound is large."""
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, dim)) * 1e-3
    for r in range(n):
        idx = rng.choice(dim, size=rng.integers(1, 5), replace=False)
        x[r, idx] = rng.standard_normal(idx.size)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    return _to_u16(x)


def test_scan_form_by_k(gpu, oracle_mod):
    from audio_rag_amd import _armi

    idx = _index(oracle_mod.unit_fp16(500, 1024, seed=1), gpu)
    assert idx.scan_form(64, 5) == _armi.SCAN_INT8_FILTER
    assert idx.scan_form(64, 16) == _armi.SCAN_INT8_FILTER
    assert idx.scan_form(64, 40) == _armi.SCAN_INT8_FILTER  # the reference's hybrid prefetch
    assert idx.scan_form(64, 64) == _armi.SCAN_INT8_FILTER
    assert idx.scan_form(64, 65) == _armi.SCAN_FP16
    assert idx.scan_form(300, 5) == _armi.SCAN_TILED_FP16  # < 200k rows: the fp16 tiled scan


@pytest.mark.parametrize("k", [1, 5, 6, 7, 10, 16, 17, 40, 65])
def test_filter_forms_match_oracle(gpu, oracle_mod, k):
    rows = oracle_mod.unit_fp16(30000, 1024, seed=300 + k)
    qs = oracle_mod.unit_fp16(64, 1024, seed=301 + k)
    idx = _index(rows, gpu, base=7)
    _assert_same(_run(idx, qs, k, gpu), oracle_mod.dense_topk(rows, qs, k, ordinal_base=7))


@pytest.mark.parametrize("dim", [256, 512, 768, 1024])
def test_spiky_rows_and_queries(gpu, oracle_mod, dim):
    rows = _spiky_rows(6000, dim, seed=dim)
    # queries: half spiky (aligned with some rows' spikes), half dense random
    qs = np.concatenate([_spiky_rows(32, dim, seed=dim + 1), oracle_mod.unit_fp16(32, dim, seed=dim + 2)])
    idx = _index(rows, gpu)
    for k in (5, 10):
        _assert_same(_run(idx, qs, k, gpu), oracle_mod.dense_topk(rows, qs, k))


def test_near_duplicates_zero_rows_and_mask(gpu, oracle_mod):
    """Rows that differ in one fp16 ulp (same int8 image, distinct exact keys) and exact
    duplicates (ordinal tie-break), zero rows (key 0 on both sides), and a row filter."""
    base = oracle_mod.unit_fp16(400, 1024, seed=77)
    dup = base.copy()
    dup[:, 0] = dup[:, 0] + 1  # one ulp of the first component
    rows = np.concatenate([base, dup, base[:50], np.zeros((30, 1024), np.uint16)])
    qs = np.concatenate([base[:40], oracle_mod.unit_fp16(24, 1024, seed=78)])
    idx = _index(rows, gpu, base=100)
    _assert_same(_run(idx, qs, 6, gpu), oracle_mod.dense_topk(rows, qs, 6, ordinal_base=100))
    n = rows.shape[0]
    keep = np.zeros((n + 63) // 64, dtype=np.uint64)
    for r in range(0, n, 3):
        keep[r >> 6] |= np.uint64(1) << np.uint64(r & 63)
    got = _run(idx, qs, 6, gpu, mask=keep)
    _assert_same(got, oracle_mod.dense_topk(rows, qs, 6, ordinal_base=100, row_mask=keep))


@pytest.mark.parametrize("k", [5, 10])
def test_certified_at_100k(gpu, oracle_mod, k):
    """Random unit rows: the bound is tight enough that no query needs the exact fallback."""
    from audio_rag_amd import _armi

    rows = oracle_mod.unit_fp16(100000, 1024, seed=500 + k)
    qs = oracle_mod.unit_fp16(64, 1024, seed=501 + k)
    idx = _index(rows, gpu)
    assert idx.scan_form(64, k) == _armi.SCAN_INT8_FILTER
    got = _run(idx, qs, k, gpu)
    assert (got["flags"] == 1).all(), got["flags"]
    _assert_same(got, oracle_mod.dense_topk(rows, qs, k))


def test_nontemporal_stream_first_and_collect_pass(gpu, oracle_mod):
    """A shard whose int8 image (> 192 MB) streams with nontemporal loads: the first pass and the
    collect pass run the <dim, *, true> kernel instances. The collect pass is forced: 300 one-ulp
    variants of query 0 (the scattered image order spreads them over the workgroups, so every
    list keeps them) are more than the merge rescores (kc = 64), and the rest of them, with
    upper bounds above the 5th exact key, leave query 0 uncertified. Every query equals the
    exhaustive exact scan, a sample the oracle."""
    n, dim = 262_144 + 96, 1024
    rows = oracle_mod.unit_fp16(n, dim, seed=901)
    v = rows[5].copy()
    for i in range(300):  # one-ulp variants of v (one component each)
        w = v.copy()
        w[i] = w[i] + 1
        rows[1000 + i] = w
    qs = oracle_mod.unit_fp16(64, dim, seed=902)
    qs[0] = v
    idx = _index(rows, gpu, base=7)
    assert idx.scan_nontemporal(64, 5)
    got = _run(idx, qs, 5, gpu)
    assert got["flags"][0] != 1  # query 0 went through the collect pass
    exact = idx.topk(_dev(qs.view(np.float16), gpu), 5, exact=True)
    torch.cuda.synchronize()
    for f in ("ids", "scores", "rank", "count"):
        np.testing.assert_array_equal(got[f], getattr(exact, f).cpu().numpy(), err_msg=f)
    sample = [0, 1, 63]
    ref = oracle_mod.dense_topk(rows, qs[sample], 5, ordinal_base=7)
    np.testing.assert_array_equal(got["ids"][sample], ref.ids)
    np.testing.assert_array_equal(got["scores"][sample], ref.scores)
    small = _index(rows[:100_000], gpu)
    assert not small.scan_nontemporal(64, 5)  # 100 MB image: plain loads
