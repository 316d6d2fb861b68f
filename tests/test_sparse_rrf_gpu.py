"""Sparse lexical top-k (armi_sparse_topk) and RRF fusion (armi_rrf_fuse) on the GPU against the
CPU oracle. Integer / index work: ids and counts bit-identical; sparse scores are the exact fp32
Qdrant-order sums (bitwise); RRF scores are fp64 sums (bitwise).
Reference call sites: src/audio_rag/retrieval/qdrant.py:289-293, 299-312 (sparse), 295 (RRF)."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _t(a, gpu):
    return torch.from_numpy(np.ascontiguousarray(a)).to(gpu)


def _sparse_index(csr, gpu, base=0):
    from audio_rag_amd.retrieval.device import SparseIndex

    indptr, indices, values = csr
    return SparseIndex(_t(indptr, gpu), _t(indices, gpu), _t(values, gpu), 250002, base)


def _run(idx, qcsr, k, gpu, mask=None):
    qi, qx, qv = qcsr
    m = None if mask is None else _t(mask.view(np.int64), gpu)
    out = idx.topk(_t(qi, gpu), _t(qx, gpu), _t(qv, gpu), k, row_mask=m)
    torch.cuda.synchronize()
    return {f: getattr(out, f).cpu().numpy() for f in ("ids", "scores", "count", "flags")}


def _same(got, ref):
    np.testing.assert_array_equal(got["count"], ref.count)
    for b in range(ref.count.shape[0]):
        c = ref.count[b]
        np.testing.assert_array_equal(got["ids"][b, :c], ref.ids[b, :c], err_msg=f"query {b}")
        np.testing.assert_array_equal(got["scores"][b, :c], ref.scores[b, :c], err_msg=f"query {b}")
        assert (got["ids"][b, c:] == -1).all()


@pytest.mark.parametrize("n,b,k", [(3000, 8, 5), (20000, 64, 40), (777, 70, 12), (40, 5, 20)])
def test_sparse_matches_oracle(gpu, oracle_mod, n, b, k):
    csr = oracle_mod.sparse_corpus(n, seed=2 + n)
    q = oracle_mod.sparse_queries(b, seed=3 + n)
    idx = _sparse_index(csr, gpu, base=7)
    got = _run(idx, q, k, gpu)
    _same(got, oracle_mod.sparse_topk(*csr, *q, k, ordinal_base=7))


def test_sparse_certifies_and_masks(gpu, oracle_mod):
    n = 50000
    csr = oracle_mod.sparse_corpus(n, seed=21)
    q = oracle_mod.sparse_queries(64, seed=22)
    idx = _sparse_index(csr, gpu)
    got = _run(idx, q, 40, gpu)
    assert (got["flags"] & 1).mean() > 0.9, got["flags"]
    _same(got, oracle_mod.sparse_topk(*csr, *q, 40))
    rng = np.random.default_rng(1)
    mask = np.zeros((n + 63) // 64, dtype=np.uint64)
    for r in np.nonzero(rng.random(n) < 0.5)[0]:
        mask[r >> 6] |= np.uint64(1) << np.uint64(r & 63)
    got = _run(idx, q, 10, gpu, mask=mask)
    _same(got, oracle_mod.sparse_topk(*csr, *q, 10, row_mask=mask))


def test_sparse_no_overlap_and_empty_query(gpu, oracle_mod):
    csr = oracle_mod.sparse_corpus(500, seed=31)
    qi = np.array([0, 0, 2], dtype=np.int32)           # query 0 empty, query 1 two unseen terms
    qx = np.array([250000, 250001], dtype=np.int32)
    qv = np.array([0.3, 0.2], dtype=np.float32)
    idx = _sparse_index(csr, gpu)
    got = _run(idx, (qi, qx, qv), 5, gpu)
    assert (got["count"] == 0).all()
    _same(got, oracle_mod.sparse_topk(*csr, qi, qx, qv, 5))


def _rrf_case(rng, n_q, ka, kb, universe):
    a_ids = np.full((n_q, ka), -1, dtype=np.int64)
    b_ids = np.full((n_q, kb), -1, dtype=np.int64)
    a_cnt = rng.integers(0, ka + 1, size=n_q).astype(np.int32)
    b_cnt = rng.integers(0, kb + 1, size=n_q).astype(np.int32)
    for q in range(n_q):
        a_ids[q, :a_cnt[q]] = rng.choice(universe, size=a_cnt[q], replace=False)
        b_ids[q, :b_cnt[q]] = rng.choice(universe, size=b_cnt[q], replace=False)
    return a_ids, a_cnt, b_ids, b_cnt


@pytest.mark.parametrize("ka,kb,limit,universe", [(40, 40, 20, 60), (10, 10, 5, 15), (200, 200, 100, 300), (3, 7, 20, 9)])
def test_rrf_matches_qdrant_local_mode(gpu, oracle_mod, ka, kb, limit, universe):
    from audio_rag_amd.retrieval.device import TopK, rrf_fuse

    rng = np.random.default_rng(ka * 7 + kb)
    a_ids, a_cnt, b_ids, b_cnt = _rrf_case(rng, 33, ka, kb, universe)
    z = lambda x: _t(x, gpu)
    a = TopK(scores=None, ids=z(a_ids), rank=None, count=z(a_cnt))
    b = TopK(scores=None, ids=z(b_ids), rank=None, count=z(b_cnt))
    out = rrf_fuse(a, b, limit, rrf_k=2)
    torch.cuda.synchronize()
    ids, rank, cnt = out.ids.cpu().numpy(), out.rank.cpu().numpy(), out.count.cpu().numpy()
    for q in range(33):
        ref = oracle_mod.rrf([list(a_ids[q, :a_cnt[q]]), list(b_ids[q, :b_cnt[q]])], limit)
        assert cnt[q] == len(ref)
        assert [int(x) for x in ids[q, :cnt[q]]] == [int(p) for p, _ in ref]
        assert [float(x) for x in rank[q, :cnt[q]]] == [s for _, s in ref]


def test_sparse_empty_rows_and_long_rows(gpu, oracle_mod):
    """Rows without sparse entries (e.g. points stored dense-only) and rows longer than a 64-entry
    block, interleaved, so row boundaries fall anywhere inside the scan's entry blocks."""
    indptr, indices, values = oracle_mod.sparse_corpus(5000, seed=41)
    lens = np.diff(indptr)
    keep = np.ones(len(lens), dtype=bool)
    keep[::3] = False  # every third row empty
    new_ptr = np.zeros_like(indptr)
    np.cumsum(np.where(keep, lens, 0), out=new_ptr[1:])
    sel = np.concatenate([np.arange(indptr[r], indptr[r + 1]) for r in range(len(lens)) if keep[r]])
    csr = (new_ptr, indices[sel], values[sel])
    q = oracle_mod.sparse_queries(20, seed=42)
    idx = _sparse_index(csr, gpu)
    for k in (3, 40):
        got = _run(idx, q, k, gpu)
        _same(got, oracle_mod.sparse_topk(*csr, *q, k))
        assert not np.isin(got["ids"], np.nonzero(~keep)[0]).any()


def test_sparse_golden_corpus_repeatable(gpu, oracle_mod):
    """The golden scenario's lexical corpus (300 chunks over a 600-id vocabulary slice: every
    posting list is short, so every cursor comes from the in-list search), single queries and
    batches, with and without metadata filters, each search run three times."""
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))
    import replay
    import scenario

    s = scenario.build()
    csr = replay.corpus_csr(s, True)
    idx = _sparse_index(csr, gpu)
    nq = len(s["qlex"])
    parts = [replay.query_csr(s, q) for q in range(nq)]
    qi = np.zeros(nq + 1, np.int32)
    np.cumsum([len(p[1]) for p in parts], out=qi[1:])
    batch = (qi, np.concatenate([p[1] for p in parts]), np.concatenate([p[2] for p in parts]))
    masks = [None] + [replay.filter_mask(s, {"lecture": v}) for v in range(3)]
    for mask in masks:
        for k in (10, 20, 40):
            want = oracle_mod.sparse_topk(*csr, *batch, k, row_mask=mask)
            for _ in range(3):
                _same(_run(idx, batch, k, gpu, mask=mask), want)
            for q in range(0, nq, 7):
                one = parts[q]
                want1 = oracle_mod.sparse_topk(*csr, *one, k, row_mask=mask)
                for _ in range(3):
                    _same(_run(idx, one, k, gpu, mask=mask), want1)


def test_sparse_pass_with_many_distinct_terms(gpu, oracle_mod):
    """64 queries x 200 distinct corpus terms, disjoint across queries: one pass holds 12 800
    distinct terms, i.e. 100 staging segments of 128 terms (more segments than wave lanes)."""
    csr = oracle_mod.sparse_corpus(20000, seed=51)
    rng = np.random.default_rng(52)
    nq, nt = 64, 200
    present = np.unique(csr[1])
    assert present.size >= nq * nt
    # ascending within each query, as the host layer hands query CSRs to the device (and the
    # oracle's merge-join expects)
    qx = np.sort(rng.permutation(present)[:nq * nt].reshape(nq, nt), axis=1).reshape(-1).astype(np.int32)
    qi = np.arange(0, nq * nt + 1, nt, dtype=np.int32)
    qv = rng.uniform(0.05, 0.35, nq * nt).astype(np.float32)
    idx = _sparse_index(csr, gpu)
    for k in (5, 40):
        got = _run(idx, (qi, qx, qv), k, gpu)
        _same(got, oracle_mod.sparse_topk(*csr, qi, qx, qv, k))
        assert (got["count"] > 0).all()


def test_sparse_max_k_and_several_passes(gpu, oracle_mod):
    """k = 240 (MAX_K) over 150 queries: three 64-query passes, the last one partial."""
    from audio_rag_amd.retrieval.device import MAX_K

    csr = oracle_mod.sparse_corpus(8000, seed=61)
    q = oracle_mod.sparse_queries(150, seed=62)
    idx = _sparse_index(csr, gpu, base=3)
    _same(_run(idx, q, MAX_K, gpu), oracle_mod.sparse_topk(*csr, *q, MAX_K, ordinal_base=3))


@pytest.mark.parametrize("vocab", [250002, 1 << 20])
def test_sparse_pass_term_numbering_paths(gpu, oracle_mod, vocab):
    """A pass numbers its distinct terms by an LDS bitmap when vocab <= 2^18 (BGE-M3) and by a
    sort otherwise (pass_terms_bitmap_kernel / pass_terms_kernel): both give the oracle's answer.
    With vocab = 2^20 the ids >= 200 000 are moved up by 300 000 (an order-preserving map, so
    every query stays ascending), so terms live above the bitmap's range too."""
    from audio_rag_amd.retrieval.device import SparseIndex

    indptr, indices, values = oracle_mod.sparse_corpus(6000, seed=71)
    qi, qx, qv = oracle_mod.sparse_queries(64, seed=72)
    if vocab > 250002:
        indices = np.where(indices >= 200000, indices + 300000, indices).astype(np.int32)
        qx = np.where(qx >= 200000, qx + 300000, qx).astype(np.int32)
    idx = SparseIndex(_t(indptr, gpu), _t(indices, gpu), _t(values, gpu), vocab, 5)
    for k in (3, 20):
        want = oracle_mod.sparse_topk(indptr, indices, values, qi, qx, qv, k, ordinal_base=5)
        _same(_run(idx, (qi, qx, qv), k, gpu), want)


def _overflow_corpus(n=200_000, pile=6000, t_rows=5000, seed=81):
    """n rows of 8 stratified terms (ascending, < 50 000) with U(0.01, 0.40) values; even rows
    also hold term 60 000 (a dense value column: present in half the rows); rows [0, t_rows) hold
    term 70 000 with a value from {0.1, 0.2, 0.3} (many ties); rows 0, 20, 40, ... (pile of them)
    copy row 0's first nine entries exactly (a pile of re-uploaded identical chunks)."""
    rng = np.random.default_rng(seed)
    base = (rng.integers(0, 6250, size=(n, 8)) + 6250 * np.arange(8)).astype(np.int32)
    bval = rng.uniform(0.01, 0.40, size=(n, 8)).astype(np.float32)
    even = (np.arange(n) % 2 == 0)
    tee = np.arange(n) < t_rows
    p_rows = np.arange(pile) * 20
    base[p_rows] = base[0]
    bval[p_rows] = bval[0]
    dval = rng.uniform(0.01, 0.40, size=n).astype(np.float32)
    dval[p_rows] = dval[0]
    tval = rng.choice(np.array([0.1, 0.2, 0.3], np.float32), size=n)
    lens = 8 + even.astype(np.int64) + tee.astype(np.int64)
    indptr = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=indptr[1:])
    indices = np.empty(indptr[-1], np.int32)
    values = np.empty(indptr[-1], np.float32)
    cols = np.arange(8)
    pos = indptr[:-1, None] + cols
    indices[pos.ravel()] = base.ravel()
    values[pos.ravel()] = bval.ravel()
    e = np.nonzero(even)[0]
    indices[indptr[e] + 8] = 60000
    values[indptr[e] + 8] = dval[e]
    t = np.nonzero(tee)[0]
    at = indptr[t] + 8 + even[t].astype(np.int64)
    indices[at] = 70000
    values[at] = tval[t]
    return (indptr, indices, values), p_rows


def test_sparse_collect_overflow_is_exact(gpu, oracle_mod):
    """More than kCollectCap = 4096 rows reach the collect threshold: (a) a pile of 6 000
    identical rows tying at the top (the k-th candidate's score is the pile's), (b) a query whose
    one term lies in rows [0, 5 000) only, so at k = 240 the merge pools fewer than k candidates
    (threshold -inf: every overlapping row is collected). The helper workgroups of the collect
    merge must answer both exactly (ids by ascending ordinal among ties), filtered and not."""
    csr, p_rows = _overflow_corpus()
    indptr, indices, values = csr
    rng = np.random.default_rng(82)
    r0 = slice(indptr[0], indptr[0] + 9)  # row 0: 8 base terms + the dense-column term
    pile_q = (indices[r0], rng.uniform(0.05, 0.35, 9).astype(np.float32))
    tee_q = (np.array([70000], np.int32), np.array([0.3], np.float32))
    mixed = oracle_mod.sparse_queries(6, seed=83)
    parts = [pile_q, tee_q] + [(mixed[1][mixed[0][i]:mixed[0][i + 1]],
                                mixed[2][mixed[0][i]:mixed[0][i + 1]]) for i in range(6)]
    qi = np.zeros(len(parts) + 1, np.int32)
    np.cumsum([len(p[0]) for p in parts], out=qi[1:])
    q = (qi, np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]))
    idx = _sparse_index(csr, gpu, base=11)
    n = indptr.size - 1
    mask = np.zeros((n + 63) // 64, dtype=np.uint64)
    for r in np.nonzero(rng.random(n) < 0.5)[0]:
        mask[r >> 6] |= np.uint64(1) << np.uint64(r & 63)
    for k in (5, 40, 240):
        for m in (None, mask):
            got = _run(idx, q, k, gpu, mask=m)
            _same(got, oracle_mod.sparse_topk(*csr, *q, k, row_mask=m, ordinal_base=11))
            # the pile and the -inf-threshold queries are never answered by the MFMA filter
            assert not (got["flags"][:2] & 4).any(), got["flags"]
            # the pile query always needs the overflow path
            assert got["flags"][0] & 2, got["flags"]
            if m is None:
                np.testing.assert_array_equal(got["ids"][0, :k], p_rows[:k] + 11)
    # the -inf threshold case: 5 000 overlapping rows in <= 7 ranges pool < 240 candidates
    got = _run(idx, q, 240, gpu)
    assert got["flags"][1] & 2 and got["count"][1] == 240


def test_sparse_zero_negative_and_denormal_products(gpu, oracle_mod):
    """Products that are not normal positive floats keep the oracle's answer: a pass with one
    zero and one negative weight, a pass whose products underflow to denormals, and an index
    holding zero values (rows sharing only a zero-valued term are still results, score 0)."""
    csr = oracle_mod.sparse_corpus(20000, seed=91)
    qi, qx, qv = oracle_mod.sparse_queries(64, seed=92)
    idx = _sparse_index(csr, gpu)
    for k in (5, 40):
        _same(_run(idx, (qi, qx, qv), k, gpu), oracle_mod.sparse_topk(*csr, qi, qx, qv, k))
    odd = qv.copy()
    odd[qi[3]] = 0.0
    odd[qi[9]] = -0.2
    _same(_run(idx, (qi, qx, odd), 20, gpu), oracle_mod.sparse_topk(*csr, qi, qx, odd, 20))
    tiny = (qv * np.float32(1e-37)).astype(np.float32)
    _same(_run(idx, (qi, qx, tiny), 20, gpu), oracle_mod.sparse_topk(*csr, qi, qx, tiny, 20))
    indptr, indices, values = csr
    values = values.copy()
    values[::97] = 0.0
    idx0 = _sparse_index((indptr, indices, values), gpu)
    _same(_run(idx0, (qi, qx, qv), 20, gpu),
          oracle_mod.sparse_topk(indptr, indices, values, qi, qx, qv, 20))


def _clustered_case(oracle_mod, gpu, n, rows, seed):
    """The corpus of sparse_corpus(n) with a posting-list term t (below 1/8 of the rows) added to
    `rows`, and 64 queries that all carry t: (device index, csr, query csr)."""
    indptr, indices, values = oracle_mod.sparse_corpus(n, seed=seed)
    t = 249_999  # not in the Zipf corpus's head
    add = np.zeros(n, dtype=bool)
    add[rows] = True
    new_ptr = np.zeros_like(indptr)
    np.cumsum(np.diff(indptr) + add, out=new_ptr[1:])
    ni = np.empty(new_ptr[-1], np.int32)
    nv = np.empty(new_ptr[-1], np.float32)
    rng = np.random.default_rng(seed + 1)
    for r in range(n):
        a, b = indptr[r], indptr[r + 1]
        c = new_ptr[r]
        ids, vals = indices[a:b], values[a:b]
        if add[r]:
            keep = ids != t
            ids = np.append(ids[keep], t)
            vals = np.append(vals[keep], np.float32(rng.uniform(0.01, 0.4)))
            o = np.argsort(ids, kind="stable")
            ids, vals = ids[o], vals[o]
        ni[c:c + len(ids)] = ids
        nv[c:c + len(ids)] = vals
    csr = (new_ptr, ni, nv)
    qi, qx, qv = oracle_mod.sparse_queries(64, seed=seed + 2)
    # every query also carries t (kept ascending)
    xs, vs = [], []
    for b in range(64):
        x, v = qx[qi[b]:qi[b + 1]], qv[qi[b]:qi[b + 1]]
        keep = x != t
        x, v = np.append(x[keep], t), np.append(v[keep], np.float32(0.3))
        o = np.argsort(x, kind="stable")
        xs.append(x[o])
        vs.append(v[o])
    qx2 = np.concatenate(xs).astype(np.int32)
    qv2 = np.concatenate(vs).astype(np.float32)
    qi2 = np.zeros(65, np.int32)
    np.cumsum([len(x) for x in xs], out=qi2[1:])
    return _sparse_index(csr, gpu), csr, (qi2, qx2, qv2)


def test_sparse_clustered_postings(gpu, oracle_mod):
    """A posting-list term (below 1/8 of the rows) whose postings fill whole tiles, so the scan's
    staged window of 128 postings is entirely inside the tile (its next posting row is only
    bounded, not read) and the following tiles start from the advanced cursor."""
    idx, csr, q = _clustered_case(oracle_mod, gpu, 20000, np.r_[0:300, 5000:5090, 19_900:20000], 93)
    for k in (5, 40):
        _same(_run(idx, q, k, gpu), oracle_mod.sparse_topk(*csr, *q, k))


def test_sparse_clustered_postings_beyond_one_load(gpu, oracle_mod):
    """200k rows (832-row ranges, so whole 256-row tiles): a posting-list term with runs of 300
    and 700 contiguous rows, i.e. more postings inside one tile than one 128-posting load holds
    (the scan reloads 128 at a time, round 5), plus runs across range and tile edges."""
    rows = np.r_[0:300, 800:870, 50_000:50_700, 123_456:123_700, 199_700:200_000]
    idx, csr, q = _clustered_case(oracle_mod, gpu, 200_000, rows, 193)
    for k in (5, 40):
        _same(_run(idx, q, k, gpu), oracle_mod.sparse_topk(*csr, *q, k))
