"""QueryBatcher on the GPU: answers coalesced from concurrent callers equal what
MI355XRetriever.search returns for each query alone (dense, sparse and hybrid, with and
without a metadata filter)."""

import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_batched_answers_equal_single_searches(gpu, oracle_mod):
    from audio_rag_amd.config import RetrievalConfig
    from audio_rag_amd.core import EmbeddingResult, SparseVector
    from audio_rag_amd.retrieval.batcher import QueryBatcher
    from audio_rag_amd.retrieval.mi355x import MI355XRetriever

    n = 4000
    rows = oracle_mod.unit_fp16(n, 1024, seed=51).view(np.float16)
    csr = oracle_mod.sparse_corpus(n, seed=52)
    sparse = [(csr[1][csr[0][i]:csr[0][i + 1]], csr[2][csr[0][i]:csr[0][i + 1]]) for i in range(n)]
    payloads = [{"text": f"c{i}", "start": i, "end": i + 1, "speaker": None,
                 "metadata": {"lecture": i % 3}} for i in range(n)]
    ret = MI355XRetriever(RetrievalConfig(top_k=7), 1024)
    ret.add_arrays(rows, payloads, sparse=sparse)
    qi, qx, qv = oracle_mod.sparse_queries(90, seed=53)
    qd = oracle_mod.unit_fp16(90, 1024, seed=54).view(np.float16).astype(np.float32)
    queries = [EmbeddingResult(dense=qd[i].tolist(),
                               sparse=SparseVector(qx[qi[i]:qi[i + 1]].tolist(),
                                                   qv[qi[i]:qi[i + 1]].tolist()) if i % 4 else None)
               for i in range(90)]
    filters = [None if i % 5 else {"lecture": i % 3} for i in range(90)]
    for st in ("hybrid", "dense", "sparse"):
        want = [ret.search(q, filter_metadata=f, search_type=st) for q, f in zip(queries, filters)]
        got = [None] * 90
        with QueryBatcher(ret, search_type=st, max_batch=32, max_wait_ms=5.0) as qb:
            def client(lo):
                for i in range(lo, 90, 3):
                    got[i] = qb.submit(queries[i], filters[i])
            ts = [threading.Thread(target=client, args=(c,)) for c in range(3)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            got = [f.result(timeout=60) for f in got]
            assert qb.batches < 90
        for i in range(90):
            assert [(r.chunk.text, r.score, r.source) for r in got[i]] == \
                   [(r.chunk.text, r.score, r.source) for r in want[i]], (st, i)
