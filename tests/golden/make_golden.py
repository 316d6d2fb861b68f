"""Generates tests/golden/reference_query_path.json by running the REFERENCE's own query-path
code (/root/reference/src: AudioRAG, QueryPipeline, QdrantRetriever, BGEM3Embedder, BGEReranker)
on the seeded inputs of scenario.py.

Only the third-party engines the reference delegates to are replaced, because none is installed
(SURVEY.md §8(c)): qdrant_client (an in-memory store restating qdrant-client local mode: COSINE
normalise-at-insert + fp32 dot, fp32 sparse dot over shared indices, RRF 1/(2+pos) with a stable
sort, MatchValue filters, score_threshold, upsert = overwrite), FlagEmbedding.BGEM3FlagModel
(returns the scenario's vectors) and sentence_transformers.CrossEncoder (returns the scenario's
scores; raises for one query). Every engine call is recorded in the fixture's trace.

Run in the build container (the reference is not on the GPU box):
    python tests/golden/make_golden.py
"""

from __future__ import annotations

import json
import sys
import types
from collections import defaultdict
from dataclasses import dataclass, field
from enum import Enum
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
import scenario  # noqa: E402

REF_SRC = "/root/reference/src"
REF_CONFIGS = "/root/reference/configs"
S = scenario.build()
TRACE: list[dict] = []
TEXT2DENSE = {t: S["dense"][i] for i, t in enumerate(S["chunk_texts"])}
TEXT2LEX = {t: S["lex"][i] for i, t in enumerate(S["chunk_texts"])}
for q, t in enumerate(S["query_texts"]):
    TEXT2DENSE[t] = S["qdense"][q]
    TEXT2LEX[t] = S["qlex"][q]


# --------------------------------------------------------------------- fake qdrant_client

class Distance(str, Enum):
    COSINE = "Cosine"


class Fusion(str, Enum):
    RRF = "rrf"


@dataclass
class VectorParams:
    size: int
    distance: Distance


@dataclass
class SparseIndexParams:
    on_disk: bool | None = None


@dataclass
class SparseVectorParams:
    index: SparseIndexParams | None = None


@dataclass
class SparseVector:
    indices: list
    values: list


@dataclass
class PointStruct:
    id: object
    vector: object
    payload: dict | None = None


@dataclass
class MatchValue:
    value: object


@dataclass
class FieldCondition:
    key: str
    match: MatchValue


@dataclass
class Filter:
    must: list = field(default_factory=list)


@dataclass
class Prefetch:
    query: object
    using: str | None = None
    limit: int = 10


@dataclass
class FusionQuery:
    fusion: Fusion


@dataclass
class ScoredPoint:
    id: object
    score: float
    payload: dict


def _normalize(v) -> np.ndarray:
    a = np.asarray(v, dtype=np.float32)
    n = np.linalg.norm(a)
    return a / (n if n != 0 else np.float32(1e-12))


class _Collection:
    def __init__(self, name, vectors_config, sparse_vectors_config):
        self.name = name
        self.named = isinstance(vectors_config, dict)
        self.sparse_names = list((sparse_vectors_config or {}).keys())
        self.points: dict = {}  # id -> (vectors dict, payload); dict keeps insertion order


class QdrantClient:
    def __init__(self, location=None, host=None, port=None, **kw):
        self._cols: dict[str, _Collection] = {}
        TRACE.append({"call": "QdrantClient", "location": location, "host": host, "port": port})

    def get_collections(self):
        return types.SimpleNamespace(collections=[types.SimpleNamespace(name=n) for n in self._cols])

    def create_collection(self, collection_name, vectors_config, sparse_vectors_config=None):
        named = isinstance(vectors_config, dict)
        TRACE.append({"call": "create_collection", "collection": collection_name,
                      "dense": (sorted(vectors_config) if named else "<unnamed>"),
                      "dense_size": (vectors_config["dense"].size if named else vectors_config.size),
                      "distance": (vectors_config["dense"].distance.value if named else vectors_config.distance.value),
                      "sparse": sorted((sparse_vectors_config or {}).keys())})
        self._cols[collection_name] = _Collection(collection_name, vectors_config, sparse_vectors_config)

    def get_collection(self, name):
        c = self._cols[name]
        params = types.SimpleNamespace(sparse_vectors=({n: None for n in c.sparse_names} or None))
        return types.SimpleNamespace(config=types.SimpleNamespace(params=params),
                                     points_count=len(c.points))

    def delete_collection(self, collection_name):
        TRACE.append({"call": "delete_collection", "collection": collection_name})
        self._cols.pop(collection_name, None)

    def upsert(self, collection_name, points):
        c = self._cols[collection_name]
        names = []
        for p in points:
            vec = p.vector if isinstance(p.vector, dict) else {"": p.vector}
            stored = {}
            for k, v in vec.items():
                if isinstance(v, SparseVector):
                    order = np.argsort(np.asarray(v.indices), kind="stable")
                    stored[k] = (np.asarray(v.indices, dtype=np.int64)[order],
                                 np.asarray(v.values, dtype=np.float32)[order])
                else:
                    stored[k] = _normalize(v)  # COSINE: normalised at insert
            c.points[p.id] = (stored, dict(p.payload or {}))  # upsert overwrites the point
            names.append(sorted(vec.keys()))
        TRACE.append({"call": "upsert", "collection": collection_name, "points": len(points),
                      "vectors": sorted(set(tuple(n) for n in names))})

    # --- search ------------------------------------------------------------------------

    @staticmethod
    def _passes(payload, flt: Filter | None) -> bool:
        if flt is None:
            return True
        for cond in flt.must:
            key = cond.key.split(".")
            v = payload
            for part in key:
                if not isinstance(v, dict) or part not in v:
                    return False
                v = v[part]
            want = cond.match.value
            vals = v if isinstance(v, list) else [v]
            if not any((type(x) is bool) == (type(want) is bool) and x == want for x in vals):
                return False
        return True

    def _dense(self, c, query, using, limit, flt, thr=None):
        name = using or ""
        q = _normalize(query)
        scored = []
        for order, (pid, (vecs, payload)) in enumerate(c.points.items()):
            if name not in vecs or not self._passes(payload, flt):
                continue
            s = float(np.dot(vecs[name], q))  # fp32 dot (numpy)
            if thr is not None and s < thr:
                continue
            scored.append((-s, payload["metadata"]["ordinal"], pid, s, payload))
        scored.sort(key=lambda x: (x[0], x[1]))
        return [ScoredPoint(id=x[2], score=x[3], payload=x[4]) for x in scored[:limit]]

    def _sparse(self, c, query: SparseVector, using, limit, flt):
        order = np.argsort(np.asarray(query.indices), kind="stable")
        qi = np.asarray(query.indices, dtype=np.int64)[order]
        qv = np.asarray(query.values, dtype=np.float32)[order]
        scored = []
        for pid, (vecs, payload) in c.points.items():
            if using not in vecs or not self._passes(payload, flt):
                continue
            di, dv = vecs[using]
            s = np.float32(0.0)
            hit = False
            i = j = 0
            while i < len(di) and j < len(qi):  # merge join, ascending index, fp32
                if di[i] == qi[j]:
                    s = np.float32(s + np.float32(dv[i] * qv[j]))
                    hit = True
                    i += 1
                    j += 1
                elif di[i] < qi[j]:
                    i += 1
                else:
                    j += 1
            if hit:
                scored.append((-float(s), payload["metadata"]["ordinal"], pid, float(s), payload))
        scored.sort(key=lambda x: (x[0], x[1]))
        return [ScoredPoint(id=x[2], score=x[3], payload=x[4]) for x in scored[:limit]]

    def query_points(self, collection_name, query=None, using=None, prefetch=None, limit=10,
                     query_filter=None, score_threshold=None):
        c = self._cols[collection_name]
        TRACE.append({"call": "query_points", "collection": collection_name,
                      "using": using, "limit": limit,
                      "query": ("fusion:" + query.fusion.value if isinstance(query, FusionQuery)
                                else "sparse" if isinstance(query, SparseVector) else "dense"),
                      "prefetch": [{"using": p.using, "limit": p.limit,
                                    "query": "sparse" if isinstance(p.query, SparseVector) else "dense"}
                                   for p in (prefetch or [])],
                      "filter": ([[cd.key, cd.match.value] for cd in query_filter.must]
                                 if query_filter else None),
                      "score_threshold": score_threshold})
        if isinstance(query, FusionQuery):
            responses = []
            for p in prefetch:
                if isinstance(p.query, SparseVector):
                    responses.append(self._sparse(c, p.query, p.using, p.limit, query_filter))
                else:
                    responses.append(self._dense(c, p.query, p.using, p.limit, query_filter))
            # qdrant-client local mode reciprocal_rank_fusion
            scores: dict = {}
            pile = {}
            for resp in responses:
                for pos, sp in enumerate(resp):
                    s = 1 / (2 + pos)
                    if sp.id in scores:
                        scores[sp.id] += s
                    else:
                        pile[sp.id] = sp
                        scores[sp.id] = s
            ranked = sorted(scores.items(), key=lambda it: it[1], reverse=True)[:limit]
            pts = [ScoredPoint(id=pid, score=s, payload=pile[pid].payload) for pid, s in ranked]
        elif isinstance(query, SparseVector):
            pts = self._sparse(c, query, using, limit, query_filter)
        else:
            pts = self._dense(c, query, using, limit, query_filter, score_threshold)
        return types.SimpleNamespace(points=pts)


def install_fakes():
    qc = types.ModuleType("qdrant_client")
    qc.QdrantClient = QdrantClient
    models = types.ModuleType("qdrant_client.models")
    for obj in (Distance, Fusion, VectorParams, SparseIndexParams, SparseVectorParams, SparseVector,
                PointStruct, MatchValue, FieldCondition, Filter, Prefetch, FusionQuery, ScoredPoint):
        setattr(models, obj.__name__, obj)
    qc.models = models
    sys.modules["qdrant_client"] = qc
    sys.modules["qdrant_client.models"] = models

    fe = types.ModuleType("FlagEmbedding")

    class BGEM3FlagModel:
        def __init__(self, name, device=None, use_fp16=False):
            TRACE.append({"call": "BGEM3FlagModel", "model": name, "use_fp16": use_fp16})

        def encode(self, sentences, batch_size=32, return_dense=True, return_sparse=False,
                   return_colbert_vecs=False):
            TRACE.append({"call": "encode", "n": len(sentences), "batch_size": batch_size,
                          "return_sparse": return_sparse})
            out = {"dense_vecs": np.stack([TEXT2DENSE[s] for s in sentences])}
            if return_sparse:
                out["lexical_weights"] = [dict(TEXT2LEX[s]) for s in sentences]
            return out

    fe.BGEM3FlagModel = BGEM3FlagModel
    sys.modules["FlagEmbedding"] = fe

    st = types.ModuleType("sentence_transformers")

    class CrossEncoder:
        def __init__(self, model, max_length=None, device=None):
            TRACE.append({"call": "CrossEncoder", "model": model, "max_length": max_length})

        def predict(self, pairs, batch_size=32, show_progress_bar=False):
            TRACE.append({"call": "predict", "pairs": len(pairs), "batch_size": batch_size})
            q = S["query_texts"].index(pairs[0][0])
            if q == scenario.RERANK_FAILS:
                raise RuntimeError("simulated cross-encoder failure")
            return np.array([S["rerank"][q, S["chunk_texts"].index(t)] for _, t in pairs],
                            dtype=np.float32)

    st.CrossEncoder = CrossEncoder
    sys.modules["sentence_transformers"] = st


def compress(trace: list[dict]) -> list[dict]:
    """Run-length encodes identical consecutive trace entries."""
    out: list[dict] = []
    for t in trace:
        if out and {k: v for k, v in out[-1].items() if k != "repeat"} == t:
            out[-1]["repeat"] = out[-1].get("repeat", 1) + 1
        else:
            out.append(dict(t))
    return out


def results_json(results):
    return [{"ordinal": r.chunk.metadata["ordinal"], "score": r.score, "source": r.source,
             "text": r.chunk.text, "start": r.chunk.start, "end": r.chunk.end,
             "speaker": r.chunk.speaker} for r in results]


def main() -> None:
    install_fakes()
    sys.path.insert(0, REF_SRC)
    from audio_rag import AudioRAG
    from audio_rag.config import load_config
    from audio_rag.core import AudioChunk, EmbeddingResult, SparseVector as RefSparse

    config = load_config(env="development", config_dir=REF_CONFIGS)
    rag = AudioRAG(config)
    retriever = rag.retriever  # loads the embedder first (orchestrator.py:48-57)
    chunks = [AudioChunk(**c) for c in S["chunks"]]

    # 1. reference ingest path (embed + add): dense+sparse per point, then dense-only re-upsert
    embeddings = rag.embedder.embed([c.text for c in chunks])
    retriever.add(chunks, embeddings, collection_name="ingested")
    # 2. a hybrid collection holding sparse vectors (written straight to the engine, as a
    #    collection ingested without the re-upsert would hold them)
    client = retriever._get_client()
    client.create_collection("hybrid_real", vectors_config={"dense": VectorParams(1024, Distance.COSINE)},
                             sparse_vectors_config={"sparse": SparseVectorParams(SparseIndexParams(False))})
    pts = []
    for i, (c, e) in enumerate(zip(chunks, embeddings)):
        pts.append(PointStruct(id=f"p{i}", vector={"dense": e.dense, "sparse": SparseVector(
            e.sparse.indices, e.sparse.values)}, payload={"text": c.text, "start": c.start,
                                                          "end": c.end, "speaker": c.speaker,
                                                          "metadata": c.metadata}))
    client.upsert("hybrid_real", pts)
    # 3. a legacy dense-only collection (no sparse in any embedding)
    dense_only = [EmbeddingResult(dense=e.dense, sparse=None) for e in embeddings]
    retriever.add(chunks, dense_only, collection_name="legacy")
    ingest_trace = compress(TRACE)

    searches = []
    for coll, st, k, flt in scenario.SEARCH_CASES:
        for q, qt in enumerate(S["query_texts"]):
            emb = rag.embedder.embed_query(qt)
            TRACE.clear()
            res = retriever.search(emb, top_k=k, collection_name=coll, filter_metadata=flt,
                                   search_type=st)
            searches.append({"collection": coll, "search_type": st, "top_k": k, "filter": flt,
                             "query": q, "results": results_json(res), "trace": list(TRACE)})

    # score_threshold on a legacy dense collection (configs/production.yaml:16 uses 0.3)
    retriever.config.score_threshold = 0.02
    thresholded = []
    for q, qt in enumerate(S["query_texts"]):
        emb = rag.embedder.embed_query(qt)
        TRACE.clear()
        res = retriever.search(emb, top_k=20, collection_name="legacy", search_type="dense")
        thresholded.append({"query": q, "threshold": 0.02, "results": results_json(res),
                            "trace": list(TRACE)})
    retriever.config.score_threshold = 0.0

    pipeline = []
    for name, coll, kwargs in scenario.PIPELINE_CASES:
        for q, qt in enumerate(S["query_texts"]):
            TRACE.clear()
            r = rag.query(qt, collection_name=coll, generate_answer=False, **kwargs)
            pipeline.append({"case": name, "collection": coll, "kwargs": kwargs, "query": q,
                             "results": results_json(r.results), "reranked": r.reranked,
                             "search_type": r.search_type, "response_text": r.response_text,
                             "generated_answer": r.generated_answer, "hyde_used": r.hyde_used,
                             "trace": list(TRACE)})

    out = {
        "generator": "tests/golden/make_golden.py (reference query path run with recording fakes)",
        "reference": "/root/reference @ snapshot mounted in the build container",
        "scenario_digest": scenario.digest(S),
        "ingest_trace": ingest_trace,
        "searches": searches,
        "thresholded": thresholded,
        "pipeline": pipeline,
        "counts": {c: retriever.count(c) for c in ("ingested", "hybrid_real", "legacy")},
    }
    path = HERE / "reference_query_path.json"
    path.write_text(json.dumps(out, indent=1, sort_keys=True))
    print(f"wrote {path} ({path.stat().st_size} bytes): {len(searches)} searches, "
          f"{len(pipeline)} pipeline queries")


if __name__ == "__main__":
    main()
