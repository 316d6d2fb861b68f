"""Pins the CPU oracle against outputs of the REFERENCE's own query-path code
(tests/golden/reference_query_path.json, made by tests/golden/make_golden.py from
/root/reference with recording fakes for the absent engines).

What this pins: QdrantRetriever.search's strategy choice and request shapes (prefetch limits
2*top_k, RRF fusion, limit top_k, filters), the sparse-vector drop of QdrantRetriever.add, the
QueryPipeline / BGEReranker control flow — all computed here by oracle.py and compared with what
the reference did. Dense ids: equal outside fp32 tie-ambiguous positions; dense scores within
1e-6 (fp32 rounding of the reference's normalise-then-dot); sparse / RRF: exact."""

import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))
import replay  # noqa: E402
import scenario  # noqa: E402


@pytest.fixture(scope="module")
def golden():
    return replay.load()


def _dense_rows(s):
    return s["dense"].view(np.uint16), s["qdense"].view(np.uint16)


def oracle_search(o, s, collection, search_type, k, flt, q):
    rows, qrows = _dense_rows(s)
    hybrid = replay.COLLECTION_HYBRID[collection]
    stored_sparse = collection == "hybrid_real"  # the reference's add() drops sparse vectors
    mode = o.search_mode(search_type, hybrid, True)
    mask = replay.filter_mask(s, flt)
    csr = replay.corpus_csr(s, stored_sparse)
    qcsr = replay.query_csr(s, q)
    if collection == "empty":
        return mode, [], []
    if mode in ("dense", "legacy_dense"):
        r = o.dense_topk(rows, qrows[q:q + 1], k, row_mask=mask)
        c = r.count[0]
        return mode, list(r.ids[0, :c]), list(r.scores[0, :c]), r.rank[0, :c]
    if mode == "sparse":
        r = o.sparse_topk(*csr, *qcsr, k, row_mask=mask)
        c = r.count[0]
        return mode, list(r.ids[0, :c]), list(r.scores[0, :c])
    d = o.dense_topk(rows, qrows[q:q + 1], 2 * k, row_mask=mask)
    sp = o.sparse_topk(*csr, *qcsr, 2 * k, row_mask=mask)
    fused = o.rrf([list(d.ids[0, :d.count[0]]), list(sp.ids[0, :sp.count[0]])], k)
    return mode, [int(p) for p, _ in fused], [sc for _, sc in fused]


def check(o, got_ids, got_scores, want, mode, rank=None):
    want_ids = replay.ordinals(want)
    want_scores = [r["score"] for r in want]
    assert len(got_ids) == len(want_ids)
    if mode in ("dense", "legacy_dense"):
        amb = o.tie_ambiguous(np.asarray(rank)) if len(got_ids) else np.zeros(0, bool)
        for i, (a, b) in enumerate(zip(got_ids, want_ids)):
            assert a == b or amb[i], (i, got_ids, want_ids)
        np.testing.assert_allclose(sorted(got_scores), sorted(want_scores), rtol=0, atol=1e-6)
    else:
        assert [int(x) for x in got_ids] == want_ids
        assert [float(x) for x in got_scores] == want_scores


def test_ingest_trace_shows_reference_sparse_drop(golden):
    g, _ = golden
    trace = g["ingest_trace"]
    ups = [t for t in trace if t["call"] == "upsert" and t["collection"] == "ingested"]
    assert ups[0]["vectors"] == [["dense", "sparse"]] and ups[0]["repeat"] == scenario.N_CHUNKS
    assert ups[-1]["points"] == scenario.N_CHUNKS and ups[-1]["vectors"] == [["dense"]]


def test_searches_match_reference(oracle_mod, golden):
    g, s = golden
    for case in g["searches"]:
        out = oracle_search(oracle_mod, s, case["collection"], case["search_type"],
                            case["top_k"], case["filter"], case["query"])
        mode = out[0]
        check(oracle_mod, out[1], out[2], case["results"], mode, out[3] if len(out) > 3 else None)
        (tr,) = case["trace"]
        assert tr["limit"] == case["top_k"]
        if mode == "hybrid":
            assert tr["query"] == "fusion:rrf"
            assert [p["limit"] for p in tr["prefetch"]] == [2 * case["top_k"]] * 2
            assert [p["using"] for p in tr["prefetch"]] == ["dense", "sparse"]
        else:
            assert tr["prefetch"] == [] and tr["query"] == ("sparse" if mode == "sparse" else "dense")
        want_filter = [[f"metadata.{k}", v] for k, v in (case["filter"] or {}).items()] or None
        assert tr["filter"] == want_filter


def test_thresholded_legacy_search(oracle_mod, golden):
    g, s = golden
    rows, qrows = _dense_rows(s)
    for case in g["thresholded"]:
        r = oracle_mod.dense_topk(rows, qrows[case["query"]:case["query"] + 1], 20)
        keep = [(int(i), float(sc)) for i, sc in zip(r.ids[0], r.scores[0]) if sc >= case["threshold"]]
        assert [i for i, _ in keep] == replay.ordinals(case["results"])
        assert case["trace"][0]["score_threshold"] == case["threshold"]


def test_pipeline_matches_reference(oracle_mod, golden):
    g, s = golden
    for case in g["pipeline"]:
        kw = case["kwargs"]
        plan = oracle_mod.plan_query(kw.get("top_k"), kw.get("search_type"),
                                     kw.get("enable_reranking", True), True)
        st = plan["search"]["search_type"]
        out = oracle_search(oracle_mod, s, case["collection"], st, plan["search"]["top_k"],
                            kw.get("filter_metadata"), case["query"])
        ids, scores = out[1], out[2]
        assert case["search_type"] == st
        if plan["rerank"] is None or not ids:
            assert not case["reranked"]
            want = list(zip(ids, scores))
        else:
            assert case["reranked"]
            model = None if case["query"] == scenario.RERANK_FAILS else \
                [s["rerank"][case["query"], i] for i in ids]
            ranked = oracle_mod.rerank_rules(scores, model, plan["rerank"]["top_k"],
                                             model_raises=case["query"] == scenario.RERANK_FAILS)
            want = [(ids[i], sc) for i, sc in ranked]
            # the reranker drops `source` on rescored results only
            rescored = len(ids) > plan["rerank"]["top_k"] and case["query"] != scenario.RERANK_FAILS
            assert all((r["source"] is None) == rescored for r in case["results"])
        assert [i for i, _ in want] == replay.ordinals(case["results"])
        np.testing.assert_allclose([sc for _, sc in want], [r["score"] for r in case["results"]],
                                   rtol=0, atol=1e-6)
