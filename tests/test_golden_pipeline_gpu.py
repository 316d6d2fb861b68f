"""Replays the reference's own query-path outputs (tests/golden/reference_query_path.json)
through this package on the GPU: AudioRAG -> QueryPipeline -> MI355XRetriever (libarmi dense /
sparse / RRF kernels) -> BGEReranker rules. The embedder and the cross-encoder are table-driven
doubles fed the same vectors and scores the reference's engines were fed."""

import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))
import replay  # noqa: E402
import scenario  # noqa: E402

pytestmark = pytest.mark.gpu


def _build(golden_s):
    import torch

    from audio_rag_amd import AudioRAG
    from audio_rag_amd.config import AudioRAGConfig, RetrievalConfig
    from audio_rag_amd.core import AudioChunk, BaseEmbedder, EmbeddingResult, SparseVector
    from audio_rag_amd.reranking.bge import BGEReranker

    s = golden_s
    text2q = {t: q for q, t in enumerate(s["query_texts"])}
    text2c = {t: i for i, t in enumerate(s["chunk_texts"])}

    def emb(dense_row, lex):
        sv = SparseVector(indices=[int(k) for k in lex], values=[float(v) for v in lex.values()]) if lex else None
        return EmbeddingResult(dense=[float(x) for x in dense_row.astype(np.float32)], sparse=sv)

    class TableEmbedder(BaseEmbedder):
        loaded = False
        def embed(self, texts):
            return [emb(s["dense"][text2c[t]], s["lex"][text2c[t]]) for t in texts]
        def embed_query(self, query):
            q = text2q[query]
            return emb(s["qdense"][q], s["qlex"][q])
        def load(self):
            self.loaded = True
        def unload(self):
            self.loaded = False
        is_loaded = property(lambda self: self.loaded)
        vram_required = property(lambda self: 0.0)
        dimension = property(lambda self: 1024)

    class TableReranker(BGEReranker):
        def load(self):
            self._is_loaded = True
        def score_pairs(self, query, texts):
            q = text2q[query]
            if q == scenario.RERANK_FAILS:
                raise RuntimeError("simulated cross-encoder failure")
            return [float(s["rerank"][q, text2c[t]]) for t in texts]

    # the configuration a reference deployment loads (its own loader on its own config files,
    # tests/golden/reference_config_development.json): backend "qdrant", every MI355X knob at its
    # default (reproduce_sparse_drop included)
    cfg = AudioRAGConfig(**replay.reference_config())
    assert cfg.retrieval.backend == "qdrant" and cfg.retrieval == RetrievalConfig(
        **replay.reference_config()["retrieval"])
    rag = AudioRAG(cfg)
    rag._embedder = TableEmbedder()
    retriever = rag.retriever
    pipe = rag.query_pipeline
    pipe._reranker = TableReranker(cfg.reranking, device=torch.device("cuda", 0))
    pipe._reranker_created = True
    chunks = [AudioChunk(**c) for c in s["chunks"]]
    embeddings = rag.embedder.embed([c.text for c in chunks])
    retriever.add(chunks, embeddings, collection_name="ingested")   # sparse dropped as reference
    payloads = [{"text": c.text, "start": c.start, "end": c.end, "speaker": c.speaker,
                 "metadata": c.metadata} for c in chunks]
    retriever.add_arrays(s["dense"], payloads, [replay.sorted_sparse(x) for x in s["lex"]],
                         collection_name="hybrid_real")
    retriever.add([AudioChunk(**c) for c in s["chunks"]],
                  [EmbeddingResult(dense=e.dense, sparse=None) for e in embeddings],
                  collection_name="legacy")
    return rag


@pytest.fixture(scope="module")
def setup(gpu):
    g, s = replay.load()
    return g, s, _build(s)


def _check(o, got, want, dense_like, qdense, rows):
    got_ids = [r.chunk.metadata["ordinal"] for r in got]
    want_ids = replay.ordinals(want)
    assert len(got_ids) == len(want_ids)
    if dense_like and got_ids:
        key, _ = o.dense_keys(rows, qdense, np.array(got_ids))
        amb = o.tie_ambiguous(key)
        assert all(a == b or amb[i] for i, (a, b) in enumerate(zip(got_ids, want_ids)))
        np.testing.assert_allclose([r.score for r in got], [r["score"] for r in want], rtol=0, atol=1e-6)
    else:
        assert got_ids == want_ids
        assert [r.score for r in got] == [r["score"] for r in want]
    assert [r.source for r in got] == [r["source"] for r in want]
    assert [(r.chunk.text, r.chunk.start, r.chunk.end, r.chunk.speaker) for r in got] == \
        [(r["text"], r["start"], r["end"], r["speaker"]) for r in want]


def test_counts(setup):
    g, s, rag = setup
    for c, n in g["counts"].items():
        assert rag.retriever.count(c) == n


def test_searches(setup, oracle_mod):
    g, s, rag = setup
    rows = s["dense"].view(np.uint16)
    for case in g["searches"]:
        q = case["query"]
        emb = rag.embedder.embed_query(s["query_texts"][q])
        got = rag.retriever.search(emb, top_k=case["top_k"], collection_name=case["collection"],
                                   filter_metadata=case["filter"], search_type=case["search_type"])
        mode = oracle_mod.search_mode(case["search_type"], replay.COLLECTION_HYBRID[case["collection"]], True)
        _check(oracle_mod, got, case["results"], mode in ("dense", "legacy_dense"),
               s["qdense"][q].view(np.uint16), rows)


def test_score_threshold(setup, oracle_mod):
    g, s, rag = setup
    rows = s["dense"].view(np.uint16)
    rag.retriever.config.score_threshold = g["thresholded"][0]["threshold"]
    try:
        for case in g["thresholded"]:
            q = case["query"]
            emb = rag.embedder.embed_query(s["query_texts"][q])
            got = rag.retriever.search(emb, top_k=20, collection_name="legacy", search_type="dense")
            _check(oracle_mod, got, case["results"], True, s["qdense"][q].view(np.uint16), rows)
    finally:
        rag.retriever.config.score_threshold = 0.0


def test_pipeline(setup, oracle_mod):
    g, s, rag = setup
    rows = s["dense"].view(np.uint16)
    for case in g["pipeline"]:
        q = case["query"]
        r = rag.query(s["query_texts"][q], collection_name=case["collection"],
                      generate_answer=False, **case["kwargs"])
        assert r.reranked == case["reranked"]
        assert r.search_type == case["search_type"]
        assert r.response_text == case["response_text"]
        assert r.generated_answer is None and not r.hyde_used
        dense_like = case["kwargs"].get("search_type") == "dense" and not case["reranked"]
        _check(oracle_mod, r.results, case["results"], dense_like, s["qdense"][q].view(np.uint16), rows)
