"""The certified MFMA filter of armi_sparse_topk (audio_rag_amd/csrc/sparse_filter.h): u8-level
upper bounds of every row's sparse score on the matrix cores, an exact rescore of the best
candidates from the CSR rows, a certificate, and the exact scan for what it cannot certify.
The answers must be bit-identical to the CPU oracle (Qdrant's fp32 ascending-index sums,
oracle/armi_oracle.c) and to the same index with the filter off, whichever path answered; the
tests force every path: certified (flag FILTERED), uncertified ties at the boundary, negative
values in the index, a negative query weight, a pass of more than 512 distinct terms, posting
terms with more than one 128-posting window per 1024-row tile, filters and several passes.
Reference: src/audio_rag/retrieval/qdrant.py:289-312 (sparse prefetch / sparse query)."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

FILTERED, CERTIFIED = 4, 1


def _t(a, gpu):
    return torch.from_numpy(np.ascontiguousarray(a)).to(gpu)


def _index(csr, gpu, base=0):
    from audio_rag_amd.retrieval.device import SparseIndex

    return SparseIndex(*(_t(a, gpu) for a in csr), 250002, base)


def _run(idx, q, k, gpu, mask=None):
    m = None if mask is None else _t(mask.view(np.int64), gpu)
    out = idx.topk(*(_t(a, gpu) for a in q), k, row_mask=m)
    torch.cuda.synchronize()
    return {f: getattr(out, f).cpu().numpy() for f in ("ids", "scores", "count", "flags")}


def _same(got, ref):
    np.testing.assert_array_equal(got["count"], ref.count)
    for b in range(ref.count.shape[0]):
        c = ref.count[b]
        np.testing.assert_array_equal(got["ids"][b, :c], ref.ids[b, :c], err_msg=f"query {b}")
        np.testing.assert_array_equal(got["scores"][b, :c], ref.scores[b, :c], err_msg=f"query {b}")
        assert (got["ids"][b, c:] == -1).all()


def _equal_runs(a, b):
    for f in ("ids", "scores", "count"):
        np.testing.assert_array_equal(a[f], b[f], err_msg=f)


def _synthetic(n, b, gpu, seed):
    """SURVEY §8(d)'s sparse law on the device (synthetic.py, the bench's corpus) + host copies."""
    from audio_rag_amd import synthetic

    csr = tuple(a.cpu().numpy() for a in synthetic.make_sparse_rows(0, n, gpu, seed=seed))
    q = tuple(a.cpu().numpy() for a in synthetic.make_sparse_queries(b, gpu, seed=seed + 1))
    return csr, q


@pytest.mark.parametrize("k", [5, 20, 40])
def test_filter_answers_bit_exact(gpu, oracle_mod, k):
    csr, q = _synthetic(200_000, 64, gpu, seed=41)
    idx = _index(csr, gpu, base=3)
    assert idx.set_filter(True)
    on = _run(idx, q, k, gpu)
    frac = ((on["flags"] & FILTERED) != 0).mean()
    assert frac >= 0.9, on["flags"]
    ref = oracle_mod.sparse_topk(*csr, *q, k, ordinal_base=3)
    _same(on, ref)
    idx.set_filter(False)
    off = _run(idx, q, k, gpu)
    assert not (off["flags"] & FILTERED).any()
    _equal_runs(on, off)


def test_filter_mask_and_several_passes(gpu, oracle_mod):
    csr, q = _synthetic(120_000, 150, gpu, seed=43)
    n = csr[0].size - 1
    rng = np.random.default_rng(5)
    mask = np.zeros((n + 63) // 64, dtype=np.uint64)
    for r in np.nonzero(rng.random(n) < 0.3)[0]:
        mask[r >> 6] |= np.uint64(1) << np.uint64(r & 63)
    idx = _index(csr, gpu)
    got = _run(idx, q, 40, gpu, mask=mask)
    assert ((got["flags"] & FILTERED) != 0).mean() >= 0.9
    _same(got, oracle_mod.sparse_topk(*csr, *q, 40, row_mask=mask))


def test_filter_ties_at_the_boundary_take_the_exact_scan(gpu, oracle_mod):
    """300 consecutive identical rows above every other row for query 0: its top 5 are the five
    lowest ordinals of the pile, but a lane list keeps 3 rows and a workgroup 16, so copies are
    dropped whose key equals the 5th score: the certificate must fail and the exact scan answer."""
    csr, q = _synthetic(60_000, 8, gpu, seed=45)
    ip, ix, iv = csr
    qi, qx, qv = q
    terms = qx[qi[0]:qi[1]]
    pile = (np.sort(terms), np.full(terms.size, 0.4, np.float32))
    rows = [(ix[ip[r]:ip[r + 1]], iv[ip[r]:ip[r + 1]]) for r in range(ip.size - 1)]
    for j in range(300):
        rows[1000 + j] = pile
    nip = np.zeros(len(rows) + 1, np.int64)
    nip[1:] = np.cumsum([r[0].size for r in rows])
    csr2 = (nip, np.concatenate([r[0] for r in rows]).astype(np.int32),
            np.concatenate([r[1] for r in rows]).astype(np.float32))
    idx = _index(csr2, gpu)
    got = _run(idx, q, 5, gpu)
    assert not (got["flags"][0] & FILTERED), got["flags"]
    assert ((got["flags"][1:] & FILTERED) != 0).mean() >= 0.5
    _same(got, oracle_mod.sparse_topk(*csr2, *q, 5))


def test_filter_off_for_negative_values_and_weights(gpu, oracle_mod):
    csr, q = _synthetic(40_000, 16, gpu, seed=47)
    # a negative query weight: that query goes to the exact scan, the others stay filtered
    qv = q[2].copy()
    qv[q[0][3]] = -0.25
    q2 = (q[0], q[1], qv)
    idx = _index(csr, gpu)
    got = _run(idx, q2, 20, gpu)
    assert not (got["flags"][3] & FILTERED)
    assert ((got["flags"] & FILTERED) != 0).sum() >= 12
    _same(got, oracle_mod.sparse_topk(*csr, *q2, 20))
    # one negative value anywhere in the index: the index cannot use the filter at all
    vals = csr[2].copy()
    vals[12345] = -0.01
    csr2 = (csr[0], csr[1], vals)
    idx2 = _index(csr2, gpu)
    assert not idx2.set_filter(True)
    got = _run(idx2, q, 20, gpu)
    assert not (got["flags"] & FILTERED).any()
    _same(got, oracle_mod.sparse_topk(*csr2, *q, 20))


def test_filter_pass_over_512_terms_takes_the_exact_scan(gpu, oracle_mod):
    csr, _ = _synthetic(30_000, 1, gpu, seed=49)
    rng = np.random.default_rng(9)
    b, per = 64, 12
    qx = np.concatenate([np.sort(rng.choice(np.arange(4, 250002), per, replace=False))
                         for _ in range(b)]).astype(np.int32)
    qx[::per] = rng.integers(4, 40, b)  # one frequent term per query: every query has hits
    qx = np.concatenate([np.sort(qx[i * per:(i + 1) * per]) for i in range(b)]).astype(np.int32)
    qi = (np.arange(b + 1) * per).astype(np.int32)
    qv = rng.uniform(0.05, 0.35, b * per).astype(np.float32)
    assert np.unique(qx).size > 512
    idx = _index(csr, gpu)
    got = _run(idx, (qi, qx, qv), 10, gpu)
    assert not (got["flags"] & FILTERED).any()
    _same(got, oracle_mod.sparse_topk(*csr, qi, qx, qv, 10))


def test_filter_posting_windows_beyond_one_per_tile(gpu, oracle_mod):
    """A posting term (df < rows / 8) whose postings are one contiguous run of rows: every
    1024-row tile of the run holds 1024 of them, eight 128-posting windows per tile."""
    n = 48_000
    rng = np.random.default_rng(11)
    rows = []
    for r in range(n):
        t = np.unique(rng.integers(10, 400, 20))
        if 9000 <= r < 14_500:
            t = np.unique(np.append(t, 7))
        rows.append((t.astype(np.int32), rng.uniform(0.01, 0.4, t.size).astype(np.float32)))
    ip = np.zeros(n + 1, np.int64)
    ip[1:] = np.cumsum([r[0].size for r in rows])
    csr = (ip, np.concatenate([r[0] for r in rows]), np.concatenate([r[1] for r in rows]))
    qi = np.array([0, 3, 5, 6], np.int32)
    qx = np.array([7, 20, 33, 7, 300, 7], np.int32)
    qv = np.array([0.9, 0.1, 0.2, 0.5, 0.3, 0.05], np.float32)
    idx = _index(csr, gpu)
    for k in (5, 40):
        got = _run(idx, (qi, qx, qv), k, gpu)
        _same(got, oracle_mod.sparse_topk(*csr, qi, qx, qv, k))
    assert ((got["flags"] & FILTERED) != 0).sum() >= 1


@pytest.mark.parametrize("vocab", [250002, 1 << 20])
def test_filter_prep_paths(gpu, oracle_mod, vocab):
    """The filter's per-pass prep reads a query's list from the pass_terms wave's registers when
    it is one 64-entry chunk of valid terms, else from the lists in memory (longer queries, a
    term id >= vocab, and every query of the sorted numbering path for vocab > 2^18): all give
    the oracle's answer, and most of them through the filter."""
    csr, q = _synthetic(80_000, 48, gpu, seed=51)
    ip, ix, iv = csr
    qi, qx, qv = q
    rng = np.random.default_rng(13)
    lists = [(qx[qi[b]:qi[b + 1]], qv[qi[b]:qi[b + 1]]) for b in range(qi.size - 1)]
    for b in range(0, 48, 6):  # 70-110 terms: two 64-entry chunks
        t = np.unique(np.concatenate([lists[(b + j) % 48][0] for j in range(8)]))[:110]
        lists[b] = (t, rng.uniform(0.05, 0.35, t.size).astype(np.float32))
    for b in range(3, 48, 12):  # one term id beyond the vocabulary
        t, w = lists[b]
        lists[b] = (np.append(t, vocab + 7).astype(np.int32), np.append(w, 0.3).astype(np.float32))
    if vocab > 250002:  # an order-preserving move of the upper ids beyond the bitmap's range
        ix = np.where(ix >= 200000, ix + 300000, ix).astype(np.int32)
        lists = [(np.where(t >= 200000, t + 300000, t).astype(np.int32), w) for t, w in lists]
    qi2 = np.zeros(len(lists) + 1, np.int32)
    qi2[1:] = np.cumsum([t.size for t, _ in lists])
    qx2 = np.concatenate([t for t, _ in lists]).astype(np.int32)
    qv2 = np.concatenate([w for _, w in lists]).astype(np.float32)
    csr2 = (ip, ix, iv)
    from audio_rag_amd.retrieval.device import SparseIndex

    idx = SparseIndex(*(_t(a, gpu) for a in csr2), vocab, 0)
    got = _run(idx, (qi2, qx2, qv2), 20, gpu)
    _same(got, oracle_mod.sparse_topk(*csr2, qi2, qx2, qv2, 20))
    assert ((got["flags"] & FILTERED) != 0).mean() >= 0.75, got["flags"]


def test_filter_rare_tables_with_overflow_chains(gpu, oracle_mod, monkeypatch):
    """The rescore's rare-term values come from per-term two-choice hash tables; built at 32
    postings per 8-slot bucket (ARMI_RARE_DIV) nearly every bucket pair is full and most values
    sit in the overflow chains: the answers must not change."""
    monkeypatch.setenv("ARMI_RARE_DIV", "32")
    csr, q = _synthetic(120_000, 64, gpu, seed=53)
    idx = _index(csr, gpu)
    for k in (5, 40):
        got = _run(idx, q, k, gpu)
        _same(got, oracle_mod.sparse_topk(*csr, *q, k))
        assert ((got["flags"] & FILTERED) != 0).mean() >= 0.9
