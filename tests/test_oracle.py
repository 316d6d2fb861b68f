"""The CPU oracle against independent brute-force restatements (numpy / pure Python) on small
inputs, and against the reference-shaped fp32 arithmetic (qdrant-client local mode)."""

import math

import numpy as np
import pytest


def brute_dense(rows, qs, k):
    x = rows.view(np.float16).astype(np.float64) * 2.0**24
    q = qs.view(np.float16).astype(np.float64) * 2.0**24
    xi, qi = x.astype(np.int64), q.astype(np.int64)
    dots = qi @ xi.T                       # exact int64 (|values| < 2^25, dim <= 1024)
    n2 = (xi * xi).sum(axis=1)
    inv = np.where(n2 > 0, 1.0 / np.sqrt(n2.astype(np.float64)), 0.0)
    key = dots.astype(np.float64) * inv[None, :]
    order = np.lexsort((np.arange(rows.shape[0])[None, :].repeat(qs.shape[0], 0), -key), axis=1)
    return key, order[:, :k]


@pytest.mark.parametrize("n,dim,b,k", [(300, 256, 5, 7), (1000, 1024, 3, 40), (3, 256, 2, 5)])
def test_dense_oracle_matches_bruteforce(oracle_mod, n, dim, b, k):
    rows = oracle_mod.unit_fp16(n, dim, seed=n)
    qs = oracle_mod.unit_fp16(b, dim, seed=n + 1)
    ref = oracle_mod.dense_topk(rows, qs, k)
    key, order = brute_dense(rows, qs, k)
    kk = min(k, n)
    np.testing.assert_array_equal(ref.ids[:, :kk], order[:, :kk])
    np.testing.assert_array_equal(ref.rank[:, :kk], np.take_along_axis(key, order[:, :kk], 1))
    assert (ref.count == kk).all()


def test_dense_oracle_agrees_with_fp32_local_mode(oracle_mod):
    """Outside tie-ambiguous positions the exact ranking equals qdrant local mode's fp32 one."""
    rows = oracle_mod.unit_fp16(20000, 1024, seed=5)
    qs = oracle_mod.unit_fp16(16, 1024, seed=6)
    ref = oracle_mod.dense_topk(rows, qs, 20)
    s32 = oracle_mod.dense_fp32_local(rows, qs)
    loc = oracle_mod.order_by_score(s32, 20)
    amb = oracle_mod.tie_ambiguous(ref.rank)
    assert ((ref.ids == loc) | amb).all()
    # scores: the fp32 cosine of the reference within a few fp32 ulps
    np.testing.assert_allclose(ref.scores, np.take_along_axis(s32, ref.ids, 1), rtol=0, atol=1e-6)


def test_dense_oracle_tie_break_and_mask(oracle_mod):
    rows = oracle_mod.unit_fp16(50, 256, seed=1).copy()
    rows[10] = rows[3]
    rows[40] = rows[3]
    ref = oracle_mod.dense_topk(rows, rows[3:4], 3)
    assert list(ref.ids[0]) == [3, 10, 40]
    mask = np.array([(1 << 10) | (1 << 40) | (1 << 3)], dtype=np.uint64)
    ref = oracle_mod.dense_topk(rows, rows[3:4], 5, row_mask=mask)
    assert ref.count[0] == 3 and list(ref.ids[0, :3]) == [3, 10, 40] and ref.ids[0, 3] == -1


def brute_sparse(csr, q, k):
    indptr, indices, values = csr
    qi, qx, qv = q
    out = []
    for b in range(len(qi) - 1):
        qd = dict(zip(qx[qi[b]:qi[b + 1]].tolist(), qv[qi[b]:qi[b + 1]].tolist()))
        scored = []
        for r in range(len(indptr) - 1):
            s = np.float32(0)
            hit = False
            for t, v in zip(indices[indptr[r]:indptr[r + 1]], values[indptr[r]:indptr[r + 1]]):
                if int(t) in qd:
                    s = np.float32(s + np.float32(np.float32(qd[int(t)]) * v))
                    hit = True
            if hit:
                scored.append((-float(s), r))
        scored.sort()
        out.append([r for _, r in scored[:k]])
    return out


def test_sparse_oracle_matches_bruteforce(oracle_mod):
    csr = oracle_mod.sparse_corpus(200, seed=4)
    q = oracle_mod.sparse_queries(6, seed=5)
    ref = oracle_mod.sparse_topk(*csr, *q, 8)
    bf = brute_sparse(csr, q, 8)
    for b in range(6):
        assert list(ref.ids[b, :ref.count[b]]) == bf[b]


def test_rrf_matches_documented_examples(oracle_mod):
    # Qdrant's constant: 1/(2 + pos); ties keep first-seen order (dense list first)
    out = oracle_mod.rrf([["a", "b", "c"], ["c", "d"]], limit=10)
    assert [p for p, _ in out] == ["c", "a", "b", "d"]
    assert out[0][1] == 1 / 4 + 1 / 2
    assert out[1][1] == 0.5 and out[3][1] == 1 / 3
    # 'b' (dense pos 1) and 'd' (sparse pos 1) tie at 1/3: first-seen order
    assert [p for p, _ in out][2:] == ["b", "d"]


def test_plan_query_control_flow(oracle_mod):
    assert oracle_mod.plan_query(None, None, True, True) == {
        "search": {"top_k": 20, "search_type": "hybrid"}, "rerank": {"top_k": 5}}
    assert oracle_mod.plan_query(3, None, True, True)["rerank"] == {"top_k": 3}
    assert oracle_mod.plan_query(None, "dense", False, True) == {
        "search": {"top_k": 5, "search_type": "dense"}, "rerank": None}
    assert oracle_mod.search_mode("hybrid", True, True) == "hybrid"
    assert oracle_mod.search_mode("hybrid", False, True) == "legacy_dense"
    assert oracle_mod.search_mode("sparse", True, False) == "dense"


def test_rerank_rules(oracle_mod):
    assert oracle_mod.rerank_rules([0.1, 0.3], [9, 8], top_k=5) == [(1, 0.3), (0, 0.1)]
    got = oracle_mod.rerank_rules([0.1, 0.3, 0.2], [0.5, 0.9, 0.5], top_k=2)
    assert got == [(1, 0.9), (0, 0.5)]  # stable: index 0 before index 2 on the 0.5 tie
    assert oracle_mod.rerank_rules([0.1, 0.3, 0.2], None, 2, model_raises=True) == [(1, 0.3), (2, 0.2)]


def test_delta_bound_is_rigorous_enough(oracle_mod):
    # |fp32 accumulation - exact| <= dim * 2^-24 * sum|q_i x_i| <= dim * 2^-24 * |q||x|
    assert oracle_mod.relative_delta(1024) == 4 * 1024 * math.ldexp(1, -24)
