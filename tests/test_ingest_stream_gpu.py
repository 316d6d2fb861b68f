"""configs[4] after ASR on one GPU: synthetic transcript chunks -> BGEM3Embedder.embed (24-layer
XLM-R large fp16, batch_size 32: src/audio_rag/embeddings/bge.py:104-135) -> MI355XRetriever.add
with the reference's defaults (the sparse-drop of QdrantRetriever.add, qdrant.py:183-220: the
collection is created hybrid but its points keep only the dense vector) -> the native
StreamServer under open-loop Poisson load (pipeline/ingestion.py:176-185 then per-request
search, api/v1/query.py:90-115).

Every load-generator ticket's answer must equal oracle.dense_topk over the fp16 rows embed()
produced: a hybrid request on the sparse-dropped collection fuses the dense prefetch with an
empty sparse prefetch, so its RRF order is the dense order (scores 1/(2 + pos)), and a dense
request is the dense top-k. faster-whisper (the ASR leg) is not installed and stays out of scope;
the chunks are synthetic lecture text. Seeded weights (no checkpoint offline).
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WORDS = ("gradient descent learning rate loss function model training data neural network layer "
         "weights bias optimizer batch epoch regression classification feature vector matrix "
         "probability distribution bayes kernel margin support vector tree boosting variance "
         "lecture professor example equation derivative convex objective parameter sample").split()


def test_after_asr_chain_stream_matches_oracle(gpu, oracle_mod):
    from audio_rag_amd.config.schema import AudioRAGConfig
    from audio_rag_amd.core.base import AudioChunk
    from audio_rag_amd.embeddings.bge_m3 import BGEM3Embedder
    from audio_rag_amd.retrieval.batcher import StreamServer, _sorted_terms
    from audio_rag_amd.retrieval.mi355x import MI355XRetriever

    cfg = AudioRAGConfig()
    assert cfg.retrieval.reproduce_sparse_drop and cfg.embedding.batch_size == 32
    rng = np.random.default_rng(21)
    n = 2048
    texts = [" ".join(rng.choice(WORDS, size=int(rng.integers(40, 100)))) for _ in range(n)]
    chunks = [AudioChunk(text=t, start=30.0 * i, end=30.0 * i + 30.0, speaker=f"SPEAKER_{i % 2}",
                         metadata={"lecture": i % 7}) for i, t in enumerate(texts)]
    emb = BGEM3Embedder(cfg.embedding, device=gpu)
    emb.load()
    embeddings = emb.embed(texts)
    # (the seeded sparse head gives most texts no positive lexical weight, so their sparse is
    # None, as the reference's _convert_sparse returns for an empty dict; the drop is checked below)
    assert len(embeddings) == n

    ret = MI355XRetriever(cfg.retrieval, emb.dimension)
    ret.add(chunks, embeddings)
    coll = ret.collection()
    assert coll.hybrid and coll.count == n
    assert all(s is None for s in coll.sparse_rows)  # the reference's sparse-drop
    rows = np.concatenate(coll.dense_rows).view(np.uint16)
    emitted = np.asarray([e.dense for e in embeddings], dtype=np.float32).astype(np.float16)
    np.testing.assert_array_equal(rows, emitted.view(np.uint16))  # stored = what embed() emitted

    q_texts = [" ".join(rng.choice(WORDS, size=int(rng.integers(6, 16)))) for _ in range(256)]
    q_res = emb.embed(q_texts)
    qd = np.asarray([q.dense for q in q_res], dtype=np.float32).astype(np.float16)
    # query terms: the encoder's where it emitted any, else seeded ones (so every request of the
    # hybrid server takes the hybrid branch: RRF of the dense prefetch with an empty sparse one)
    from audio_rag_amd.core.base import EmbeddingResult, SparseVector

    def _terms(q):
        if q.sparse is not None:
            return _sorted_terms(q.sparse.indices, q.sparse.values)
        idx = np.sort(rng.choice(250000, size=8, replace=False)).astype(np.int32)
        return idx, rng.uniform(0.05, 0.3, size=8).astype(np.float32)

    terms = [_terms(q) for q in q_res]
    q_res = [EmbeddingResult(dense=q.dense, sparse=SparseVector(t[0].tolist(), t[1].tolist()))
             for q, t in zip(q_res, terms)]
    with_terms = [0, 1, 2, 3]
    indptr = np.zeros(len(terms) + 1, dtype=np.int32)
    np.cumsum([t[0].size for t in terms], out=indptr[1:])
    csr = (indptr, np.concatenate([t[0] for t in terms]), np.concatenate([t[1] for t in terms]))
    k = cfg.retrieval.top_k
    want = oracle_mod.dense_topk(rows, qd.view(np.uint16), k)

    n_q = 20000
    for search_type in ("hybrid", "dense"):
        with StreamServer(ret, max_batch=64, max_wait_ms=1.0, search_type=search_type) as srv:
            lat, elapsed, ids, cnt = srv.loadgen(qd, n_q, qps=20000.0, seed=5, sparse_csr=csr,
                                                 answers=True)
            assert (lat > 0).all() and elapsed > 0
            v = np.arange(n_q) % qd.shape[0]
            np.testing.assert_array_equal(cnt, want.count[v])
            np.testing.assert_array_equal(ids, want.ids[v])
            # result objects: hybrid scores are the RRF scores of the dense order, dense ones the
            # cosines; both equal what MI355XRetriever.search returns for the same embedding
            for i in with_terms:  # queries with terms: the hybrid branch on a hybrid server
                got = srv.result(srv.submit(q_res[i]))
                ref = ret.search(q_res[i], search_type=search_type)
                assert [(r.chunk.text, r.score) for r in got] == [(r.chunk.text, r.score)
                                                                  for r in ref]
                if search_type == "hybrid":
                    assert [r.score for r in got] == [1.0 / (2 + p) for p in range(k)]
                else:
                    assert [r.score for r in got] == [float(s) for s in want.scores[i, :k]]
        print(f"{search_type}: {n_q} queries offered at 20k q/s -> {n_q / elapsed:.0f} q/s "
              f"completed, p99 {np.percentile(lat, 99) * 1e3:.2f} ms")
