"""Seeded inputs shared by tests/golden/make_golden.py (which runs the REFERENCE's own query-path
code on them) and the tests that replay them through this package. Data only: texts, fp16-exact
dense vectors, FlagEmbedding-style lexical-weight dicts and cross-encoder scores."""

from __future__ import annotations

import hashlib

import numpy as np

N_CHUNKS = 300
N_QUERIES = 10
DIM = 1024
SPEAKERS = ["SPEAKER_00", "SPEAKER_01", "SPEAKER_02", None]


def _unit_fp16(n: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, DIM), dtype=np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    return x.astype(np.float16)


def _lexical(rng: np.random.Generator, n_terms: int, pool: np.ndarray) -> dict[str, float]:
    """FlagEmbedding lexical_weights: {str(token_id): weight}, first-occurrence order (not
    sorted), weights fp16-valued."""
    ids = rng.choice(pool, size=n_terms, replace=False)
    w = rng.uniform(0.02, 0.35, size=n_terms).astype(np.float16).astype(np.float64)
    return {str(int(i)): float(v) for i, v in zip(ids, w)}


def build() -> dict:
    rng = np.random.default_rng(1234)
    pool = np.arange(4, 4 + 600)  # shared vocabulary slice so queries overlap chunks
    chunk_texts = [f"lecture chunk {i} about topic {i % 17}" for i in range(N_CHUNKS)]
    chunks = [dict(text=t, start=round(10.0 * i, 1), end=round(10.0 * i + 9.5, 1),
                   speaker=SPEAKERS[i % 4], metadata={"lecture": i % 3, "ordinal": i})
              for i, t in enumerate(chunk_texts)]
    dense = _unit_fp16(N_CHUNKS, seed=100)
    lex = [_lexical(rng, int(rng.integers(8, 40)), pool) for _ in range(N_CHUNKS)]
    query_texts = [f"what does the lecturer say about topic {q}" for q in range(N_QUERIES)]
    qdense = _unit_fp16(N_QUERIES, seed=101)
    # make query 3 a near-copy of chunk 42 so dense ranking has a clear winner
    qdense[3] = dense[42]
    qlex = [_lexical(rng, int(rng.integers(3, 12)), pool) for _ in range(N_QUERIES)]
    # cross-encoder probabilities per (query, chunk text); a few exact ties on purpose
    rerank = rng.uniform(0.0, 1.0, size=(N_QUERIES, N_CHUNKS)).astype(np.float32)
    rerank[:, 7] = rerank[:, 8]
    return dict(chunks=chunks, chunk_texts=chunk_texts, dense=dense, lex=lex,
                query_texts=query_texts, qdense=qdense, qlex=qlex, rerank=rerank)


def digest(s: dict) -> str:
    h = hashlib.sha256()
    for key in ("dense", "qdense", "rerank"):
        h.update(np.ascontiguousarray(s[key]).tobytes())
    h.update(repr(s["lex"]).encode())
    h.update(repr(s["qlex"]).encode())
    h.update(repr(s["chunks"]).encode())
    return h.hexdigest()


# ------------------------------------------------------------------------- scenario cases

SEARCH_CASES = [
    # (collection, search_type, top_k, filter)
    ("ingested", "dense", 5, None),
    ("ingested", "hybrid", 20, None),
    ("ingested", "sparse", 5, None),
    ("hybrid_real", "hybrid", 20, None),
    ("hybrid_real", "hybrid", 5, {"lecture": 1}),
    ("hybrid_real", "sparse", 10, None),
    ("hybrid_real", "dense", 7, {"lecture": 2}),
    ("legacy", "hybrid", 5, None),
]

# every pipeline case runs all queries; the cross-encoder raises for query RERANK_FAILS, so each
# case also pins the reranker's failure fallback (reranking/bge.py:143-147)
RERANK_FAILS = 9

PIPELINE_CASES = [
    # name, collection, kwargs of AudioRAG.query (generate_answer always False)
    ("default_hybrid_rerank", "hybrid_real", {}),
    ("no_rerank_dense", "hybrid_real", {"enable_reranking": False, "search_type": "dense"}),
    ("top_k_3", "hybrid_real", {"top_k": 3}),
    ("filtered", "hybrid_real", {"filter_metadata": {"lecture": 0}}),
    ("ingested_default", "ingested", {}),
    ("sparse_rerank", "hybrid_real", {"search_type": "sparse"}),
    ("empty_collection", "empty", {}),
    ("bypass_when_few", "hybrid_real", {"filter_metadata": {"ordinal": 5}}),
]
