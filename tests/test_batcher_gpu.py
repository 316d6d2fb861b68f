"""Streaming front ends on the GPU, checked against the CPU oracle (oracle/): answers that
QueryBatcher coalesces from concurrent callers (dense, sparse and hybrid, with and without a
metadata filter), and the native StreamServer (libarmi armi_stream_*: dense, concurrent callers,
its open-loop load generator). Expected results follow QdrantRetriever.search
(src/audio_rag/retrieval/qdrant.py:227-352): strategy choice, prefetch 2*top_k, RRF 1/(2+pos)
dense list first, metadata filter on both prefetches."""

import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, NQ, K = 4000, 90, 7


def _mask(n: int, keep) -> np.ndarray:
    m = np.zeros((n + 63) // 64, dtype=np.uint64)
    for r in range(n):
        if keep(r):
            m[r >> 6] |= np.uint64(1) << np.uint64(r & 63)
    return m


@pytest.fixture(scope="module")
def store(oracle_mod):
    rows = oracle_mod.unit_fp16(N, 1024, seed=51)
    csr = oracle_mod.sparse_corpus(N, seed=52)
    qi, qx, qv = oracle_mod.sparse_queries(NQ, seed=53)
    qd = oracle_mod.unit_fp16(NQ, 1024, seed=54)
    return rows, csr, (qi, qx, qv), qd


def _expected(o, store, i: int, st: str, flt) -> list[tuple[str, float]]:
    """(payload text, score) list the reference path returns for query i."""
    rows, (ip, ix, iv), (qi, qx, qv), qd = store
    mask = None if flt is None else _mask(N, lambda r: r % 3 == flt["lecture"])
    has_sparse = bool(i % 4)
    mode = o.search_mode(st, True, has_sparse)
    q1 = qd[i:i + 1]
    s_ptr = np.array([0, qi[i + 1] - qi[i]], dtype=np.int32)
    s_idx, s_val = qx[qi[i]:qi[i + 1]], qv[qi[i]:qi[i + 1]]
    if mode == "dense":
        d = o.dense_topk(rows, q1, K, row_mask=mask)
        return [(f"c{d.ids[0, j]}", float(d.scores[0, j])) for j in range(d.count[0])]
    if mode == "sparse":
        s = o.sparse_topk(ip, ix, iv, s_ptr, s_idx, s_val, K, row_mask=mask)
        return [(f"c{s.ids[0, j]}", float(s.scores[0, j])) for j in range(s.count[0])]
    d = o.dense_topk(rows, q1, 2 * K, row_mask=mask)
    s = o.sparse_topk(ip, ix, iv, s_ptr, s_idx, s_val, 2 * K, row_mask=mask)
    fused = o.rrf([d.ids[0, :d.count[0]].tolist(), s.ids[0, :s.count[0]].tolist()], K)
    return [(f"c{pid}", float(score)) for pid, score in fused]


def _retriever(store):
    from audio_rag_amd.config import RetrievalConfig
    from audio_rag_amd.retrieval.mi355x import MI355XRetriever

    rows, (ip, ix, iv), _, _ = store
    sparse = [(ix[ip[r]:ip[r + 1]], iv[ip[r]:ip[r + 1]]) for r in range(N)]
    payloads = [{"text": f"c{r}", "start": r, "end": r + 1, "speaker": None,
                 "metadata": {"lecture": r % 3}} for r in range(N)]
    ret = MI355XRetriever(RetrievalConfig(top_k=K), 1024)
    ret.add_arrays(rows.view(np.float16), payloads, sparse=sparse)
    return ret


def test_batched_answers_match_oracle(gpu, oracle_mod, store):
    from audio_rag_amd.core import EmbeddingResult, SparseVector
    from audio_rag_amd.retrieval.batcher import QueryBatcher

    ret = _retriever(store)
    _, _, (qi, qx, qv), qd = store
    qf = qd.view(np.float16).astype(np.float32)
    queries = [EmbeddingResult(dense=qf[i].tolist(),
                               sparse=SparseVector(qx[qi[i]:qi[i + 1]].tolist(),
                                                   qv[qi[i]:qi[i + 1]].tolist()) if i % 4 else None)
               for i in range(NQ)]
    filters = [None if i % 5 else {"lecture": i % 3} for i in range(NQ)]
    for st in ("hybrid", "dense", "sparse"):
        got = [None] * NQ
        with QueryBatcher(ret, search_type=st, max_batch=32, max_wait_ms=5.0) as qb:
            def client(lo):
                for i in range(lo, NQ, 3):
                    got[i] = qb.submit(queries[i], filters[i])
            ts = [threading.Thread(target=client, args=(c,)) for c in range(3)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            got = [f.result(timeout=60) for f in got]
            assert qb.batches < NQ
        for i in range(NQ):
            want = _expected(oracle_mod, store, i, st, filters[i])
            assert [(r.chunk.text, r.score) for r in got[i]] == want, (st, i)
            assert all(r.source == "audio_rag" for r in got[i])


def test_stream_server_matches_oracle(gpu, oracle_mod, store):
    """Native server: 4 caller threads submit single queries concurrently; every ticket's
    answer equals the oracle's dense top-k; the batches coalesce."""
    from audio_rag_amd.retrieval.batcher import StreamServer

    ret = _retriever(store)
    rows, _, _, qd = store
    want = oracle_mod.dense_topk(rows, qd, K)
    got = [None] * NQ
    with StreamServer(ret, max_batch=16, max_wait_ms=3.0) as srv:
        def client(lo):
            tickets = [(i, srv.submit_arrays(qd[i].view(np.float16))) for i in range(lo, NQ, 4)]
            for i, t in tickets:
                got[i] = srv.result(t)
        ts = [threading.Thread(target=client, args=(c,)) for c in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        batches, served = srv.stats()
        assert served == NQ and batches < NQ, (batches, served)
    for i in range(NQ):
        assert [r.chunk.text for r in got[i]] == [f"c{p}" for p in want.ids[i, :want.count[i]]], i
        assert [r.score for r in got[i]] == [float(s) for s in want.scores[i, :want.count[i]]], i


def test_stream_server_hybrid_matches_oracle(gpu, oracle_mod, store):
    """Native server, hybrid: queries with sparse terms (i % 4 != 0) get the RRF fusion of the
    dense and sparse 2k prefetches with fp64 RRF scores; queries without fall back to dense
    top-k (QdrantRetriever.search strategy choice, qdrant.py:253-264). Concurrent callers, one
    load-generator pass over the same CSR."""
    from audio_rag_amd.retrieval.batcher import StreamServer

    ret = _retriever(store)
    _, _, (qi, qx, qv), qd = store
    got = [None] * NQ
    with StreamServer(ret, max_batch=16, max_wait_ms=3.0, search_type="hybrid") as srv:
        def client(lo):
            tickets = []
            for i in range(lo, NQ, 3):
                sp = (qx[qi[i]:qi[i + 1]], qv[qi[i]:qi[i + 1]]) if i % 4 else None
                tickets.append((i, srv.submit_arrays(qd[i].view(np.float16), sp)))
            for i, t in tickets:
                got[i] = srv.result(t)
        ts = [threading.Thread(target=client, args=(c,)) for c in range(3)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        batches, served = srv.stats()
        assert served == NQ and batches < NQ, (batches, served)
        lat, elapsed = srv.loadgen(qd.view(np.float16), 1000, qps=20000.0, seed=4,
                                   sparse_csr=(qi, qx, qv))
        assert lat.shape == (1000,) and (lat > 0).all() and elapsed > 0
    for i in range(NQ):
        want = _expected(oracle_mod, store, i, "hybrid", None)
        assert [(r.chunk.text, r.score) for r in got[i]] == want, i


def test_stream_server_loadgen_and_filtered_edge(gpu, oracle_mod, store):
    """The native load generator completes every arrival with positive latencies; a server over
    a tiny store returns fewer than k results where the store has fewer rows."""
    from audio_rag_amd.config import RetrievalConfig
    from audio_rag_amd.retrieval.batcher import StreamServer
    from audio_rag_amd.retrieval.mi355x import MI355XRetriever

    ret = _retriever(store)
    _, _, _, qd = store
    with StreamServer(ret, max_batch=64, max_wait_ms=1.0) as srv:
        lat, elapsed = srv.loadgen(qd.view(np.float16), 3000, qps=20000.0, seed=3)
        assert lat.shape == (3000,) and (lat > 0).all() and elapsed > 0
        batches, served = srv.stats()
        assert served == 3000 and batches <= 3000
    small = MI355XRetriever(RetrievalConfig(top_k=K), 1024)
    rows3 = oracle_mod.unit_fp16(3, 1024, seed=61)
    small.add_arrays(rows3.view(np.float16), [{"text": f"s{r}", "metadata": {}} for r in range(3)])
    with StreamServer(small, max_batch=8, max_wait_ms=0.5) as srv:
        res = srv.result(srv.submit_arrays(qd[0].view(np.float16)))
    want = oracle_mod.dense_topk(rows3, qd[:1], K)
    assert want.count[0] == 3
    assert [r.chunk.text for r in res] == [f"s{p}" for p in want.ids[0, :3]]


def test_stream_server_survives_collection_delete_and_concurrent_close(gpu, oracle_mod, store):
    """Deleting the collection under an open server stops the server first (no search on a freed
    index); closing a server while another thread waits in it wakes that thread with an error
    instead of freeing the memory under it."""
    import time

    from audio_rag_amd.core.exceptions import RetrievalError
    from audio_rag_amd.retrieval.batcher import StreamServer

    ret = _retriever(store)
    _, _, _, qd = store
    srv = StreamServer(ret, max_batch=8, max_wait_ms=0.5)
    t = srv.submit_arrays(qd[0].view(np.float16))
    assert len(srv.result(t)) == K
    ret.delete_collection()
    with pytest.raises(RetrievalError):
        srv.submit_arrays(qd[1].view(np.float16))

    ret = _retriever(store)
    srv = StreamServer(ret, max_batch=64, max_wait_ms=200.0)  # the batch waits 200 ms
    t = srv.submit_arrays(qd[2].view(np.float16))
    errs = []

    def waiter():
        try:
            srv.raw_result(t, timeout=30.0)
        except RetrievalError as e:  # woken by close()
            errs.append(e)
        except Exception as e:  # noqa: BLE001 - any other failure is a test failure
            errs.append(e)

    th = threading.Thread(target=waiter)
    th.start()
    time.sleep(0.02)
    srv.close()
    th.join(10.0)
    assert not th.is_alive()
    assert len(errs) <= 1 and all(isinstance(e, RetrievalError) for e in errs)
    srv.close()  # idempotent


def test_stream_server_threshold_and_unsorted_terms(gpu, oracle_mod, store):
    """score_threshold applies to a legacy dense-only collection (qdrant.py:331) as in
    MI355XRetriever.search; sparse terms submitted in any order answer as sorted ones."""
    from audio_rag_amd.config import RetrievalConfig
    from audio_rag_amd.core import EmbeddingResult
    from audio_rag_amd.retrieval.batcher import StreamServer
    from audio_rag_amd.retrieval.mi355x import MI355XRetriever

    rows, _, (qi, qx, qv), qd = store
    legacy = MI355XRetriever(RetrievalConfig(top_k=K, score_threshold=0.05), 1024)
    legacy.add_arrays(rows.view(np.float16), [{"text": f"c{r}", "metadata": {}} for r in range(N)])
    qf = qd.view(np.float16).astype(np.float32)
    with StreamServer(legacy, max_batch=8, max_wait_ms=0.5) as srv:
        for i in range(6):
            want = legacy.search(EmbeddingResult(dense=qf[i].tolist()))
            got = srv.result(srv.submit_arrays(qd[i].view(np.float16)))
            assert [(r.chunk.text, r.score) for r in got] == [(r.chunk.text, r.score) for r in want]
            assert all(r.score >= 0.05 for r in got)
    ret = _retriever(store)
    with StreamServer(ret, max_batch=8, max_wait_ms=0.5, search_type="hybrid") as srv:
        for i in range(1, 8):
            if not i % 4:
                continue
            idx, val = qx[qi[i]:qi[i + 1]], qv[qi[i]:qi[i + 1]]
            rev = srv.result(srv.submit_arrays(qd[i].view(np.float16), (idx[::-1], val[::-1])))
            want = _expected(oracle_mod, store, i, "hybrid", None)
            assert [(r.chunk.text, r.score) for r in rev] == want, i


def test_stream_server_filters_and_search_types(gpu, oracle_mod, store):
    """Native server, per-query search_type and metadata filter (armi_stream_submit_ex): every
    branch of QdrantRetriever.search (hybrid, sparse-only, dense; the dense fallback of queries
    without terms) under the payload filter, from concurrent callers whose filters interleave
    (each change of filter closes the collecting batch). Answers equal the oracle's."""
    from audio_rag_amd.core import EmbeddingResult, SparseVector
    from audio_rag_amd.retrieval.batcher import StreamServer

    ret = _retriever(store)
    _, _, (qi, qx, qv), qd = store
    qf = qd.view(np.float16).astype(np.float32)
    queries = [EmbeddingResult(dense=qf[i].tolist(),
                               sparse=SparseVector(qx[qi[i]:qi[i + 1]].tolist(),
                                                   qv[qi[i]:qi[i + 1]].tolist()) if i % 4 else None)
               for i in range(NQ)]
    filters = [None if i % 5 else {"lecture": i % 3} for i in range(NQ)]
    types = ["hybrid", "sparse", "dense"]
    got = [None] * NQ
    with StreamServer(ret, max_batch=16, max_wait_ms=3.0, search_type="hybrid") as srv:
        def client(lo):
            tickets = [(i, srv.submit(queries[i], filters[i], types[i % 3]))
                       for i in range(lo, NQ, 3)]
            for i, t in tickets:
                got[i] = srv.result(t)
        ts = [threading.Thread(target=client, args=(c,)) for c in range(3)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        batches, served = srv.stats()
        assert served == NQ and batches < NQ, (batches, served)
        assert not srv._masks  # every filter reference released with its result
    for i in range(NQ):
        want = _expected(oracle_mod, store, i, types[i % 3], filters[i])
        assert [(r.chunk.text, r.score) for r in got[i]] == want, (i, types[i % 3], filters[i])
    with StreamServer(ret, max_batch=8, max_wait_ms=0.5) as dense_srv:
        with pytest.raises(Exception, match="needs a server"):
            dense_srv.submit(queries[1], None, "sparse")


def test_stream_server_empty_sparse_vector(gpu, oracle_mod, store):
    """A query carrying an EMPTY SparseVector takes the hybrid / sparse-only branch, as
    MI355XRetriever.search and the reference do (`if query.sparse` is true for any SparseVector
    object, qdrant.py:272/299): hybrid = RRF over the dense 2k prefetch alone (RRF scores),
    sparse-only = no results. Checked in batches with and without other queries' terms (the
    native server skips the batch's sparse pass when no query has a term)."""
    from audio_rag_amd.core import EmbeddingResult, SparseVector
    from audio_rag_amd.retrieval.batcher import StreamServer

    ret = _retriever(store)
    rows, _, (qi, qx, qv), qd = store
    qf = qd.view(np.float16).astype(np.float32)
    empty = [EmbeddingResult(dense=qf[i].tolist(), sparse=SparseVector([], [])) for i in range(6)]
    d = oracle_mod.dense_topk(rows, qd[:6], 2 * K)
    want = [[(f"c{p}", s) for p, s in oracle_mod.rrf([d.ids[i, :d.count[i]].tolist(), []], K)]
            for i in range(6)]
    for i in range(6):  # the reference path (device search, one query at a time)
        via_search = ret.search(empty[i], search_type="hybrid")
        assert [(r.chunk.text, r.score) for r in via_search] == want[i], i
        assert ret.search(empty[i], search_type="sparse") == []
    with StreamServer(ret, max_batch=8, max_wait_ms=2.0, search_type="hybrid") as srv:
        # batch 1: only empty vectors (no sparse pass); batch 2: mixed with a query with terms
        t_h = [srv.submit(empty[i], None, "hybrid") for i in range(6)]
        got_h = [srv.result(t) for t in t_h]
        t_s = [srv.submit(empty[i], None, "sparse") for i in range(3)]
        got_s = [srv.result(t) for t in t_s]
        with_terms = EmbeddingResult(dense=qf[1].tolist(),
                                     sparse=SparseVector(qx[qi[1]:qi[2]].tolist(),
                                                         qv[qi[1]:qi[2]].tolist()))
        mixed = [srv.submit(empty[i], None, "hybrid") for i in range(3)]
        t_w = srv.submit(with_terms, None, "hybrid")
        got_m = [srv.result(t) for t in mixed]
        got_w = srv.result(t_w)
    for i in range(6):
        assert [(r.chunk.text, r.score) for r in got_h[i]] == want[i], i
    assert got_s == [[], [], []]
    for i in range(3):
        assert [(r.chunk.text, r.score) for r in got_m[i]] == want[i], i
    assert [(r.chunk.text, r.score) for r in got_w] == _expected(oracle_mod, store, 1, "hybrid", None)


def test_stream_server_ring_wrap_is_detected(gpu, oracle_mod, store):
    """A caller that lets a ticket fall a whole result ring behind gets "result overwritten",
    never another ticket's results (the ring entries are published and read seqlock-style). At
    k = 240 the ring holds 2^14 tickets; 2^14 + 200 submissions wrap it."""
    from audio_rag_amd.core.exceptions import RetrievalError
    from audio_rag_amd.retrieval.batcher import StreamServer

    ret = _retriever(store)
    rows, _, _, qd = store
    k = 240
    n = (1 << 14) + 200
    with StreamServer(ret, top_k=k, max_batch=64, max_wait_ms=0.2) as srv:
        tickets = [srv.submit_arrays(qd[i % NQ].view(np.float16)) for i in range(n)]
        _, ids_last, c_last = srv.raw_result(tickets[-1])  # every earlier batch is published
        with pytest.raises(RetrievalError, match="overwritten"):
            srv.raw_result(tickets[0])
        _, ids_kept, c_kept = srv.raw_result(tickets[-(1 << 13)])
    want = oracle_mod.dense_topk(rows, qd, k)
    j_last, j_kept = (n - 1) % NQ, (n - (1 << 13)) % NQ
    assert c_last == want.count[j_last] and c_kept == want.count[j_kept]
    np.testing.assert_array_equal(ids_last[:c_last], want.ids[j_last, :c_last])
    np.testing.assert_array_equal(ids_kept[:c_kept], want.ids[j_kept, :c_kept])
