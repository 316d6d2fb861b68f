"""QueryPipeline (mirrors src/audio_rag/pipeline/query.py:35-264).

query() follows the reference line by line: final_top_k = top_k or reranking.top_k (113);
search_type default (114); HyDE (117-134); embed (137-138); with a reranker:
search(top_k=initial_k) then rerank(query_text, top_k=final_top_k) (145-160), else
search(top_k=final_top_k) (161-168); empty -> early QueryResult (170-178); response text
(181, 217-226); generation failures are warnings (185-190); any other failure ->
PipelineError (213-215).

query_batch() is the MI355X extension: B queries embedded, searched and reranked in device
batches (same per-query semantics, one kernel pass per stage instead of B).
"""

from __future__ import annotations

import logging
from dataclasses import dataclass
from pathlib import Path

import numpy as np
import torch

from audio_rag_amd.config.schema import AudioRAGConfig
from audio_rag_amd.core.base import EmbeddingResult, RetrievalResult
from audio_rag_amd.core.exceptions import PipelineError
from audio_rag_amd.embeddings import EmbeddingsRegistry
from audio_rag_amd.pipeline.components import GeneratorRegistry, HyDEExpander, ResourceManager
from audio_rag_amd.reranking import RerankerRegistry
from audio_rag_amd.retrieval import RetrievalRegistry
from audio_rag_amd.retrieval.mi355x import QueryBatch, query_sparse_arrays
from audio_rag_amd.utils.decorators import timed

logger = logging.getLogger(__name__)


@dataclass
class QueryResult:
    """query.py:20-32."""

    query: str
    collection_name: str
    results: list[RetrievalResult]
    response_text: str | None = None
    generated_answer: str | None = None
    audio_path: Path | None = None
    reranked: bool = False
    search_type: str = "dense"
    hyde_used: bool = False
    expanded_query: str | None = None


class QueryPipeline:
    def __init__(self, config: AudioRAGConfig, resource_manager: ResourceManager | None = None):
        self.config = config
        self.resource_manager = resource_manager or ResourceManager(config.resources)
        self._embedder = None
        self._retriever = None
        self._reranker = None
        self._reranker_created = False
        self._expander = None
        self._generator = None
        self._generator_created = False

    @property
    def embedder(self):
        if self._embedder is None:
            self._embedder = EmbeddingsRegistry.create(self.config.embedding.backend,
                                                       config=self.config.embedding)
        return self._embedder

    @property
    def retriever(self):
        if self._retriever is None:
            if not self.embedder.is_loaded:
                self.embedder.load()
            self._retriever = RetrievalRegistry.create(self.config.retrieval.backend,
                                                       config=self.config.retrieval,
                                                       embedding_dim=self.embedder.dimension)
        return self._retriever

    @property
    def reranker(self):
        if not self._reranker_created:
            self._reranker = RerankerRegistry.create(self.config.reranking.backend,
                                                     config=self.config.reranking)
            self._reranker_created = True
        return self._reranker

    def _get_expander(self) -> HyDEExpander | None:
        if self._expander is None:
            self._expander = HyDEExpander(config=self.config.generation)
        return self._expander

    @property
    def generator(self):
        if not self._generator_created:
            self._generator = GeneratorRegistry.create(self.config.generation.backend,
                                                       config=self.config.generation)
            self._generator_created = True
        return self._generator

    @timed
    def query(self, query_text: str, collection_name: str | None = None, top_k: int | None = None,
              filter_metadata: dict | None = None, search_type: str | None = None,
              enable_hyde: bool | None = None, enable_reranking: bool = True,
              generate_answer: bool = True, generate_audio: bool = False,
              audio_output_path: Path | str | None = None) -> QueryResult:
        resolved_collection = collection_name or self.config.retrieval.collection_name
        final_top_k = top_k or self.config.reranking.top_k
        search_type = search_type or self.config.retrieval.search_type
        use_hyde = enable_hyde if enable_hyde is not None else (self.config.expansion.backend == "hyde")
        logger.info(f"Query: '{query_text[:50]}...' -> {resolved_collection} ({search_type}, hyde={use_hyde})")
        try:
            expanded_query = None
            hyde_used = False
            embed_text = query_text
            if use_hyde:
                expander = self._get_expander()
                if expander is not None and expander.is_available:
                    expanded_query = expander.expand_single(query_text)
                    if expanded_query and expanded_query != query_text:
                        embed_text = expanded_query
                        hyde_used = True

            self.resource_manager.ensure_vram(self.embedder.vram_required)
            query_embedding: EmbeddingResult = self.embedder.embed_query(embed_text)

            reranked = False
            if enable_reranking and self.reranker is not None:
                initial_k = self.config.reranking.initial_k
                results = self.retriever.search(query_embedding, top_k=initial_k,
                                                collection_name=resolved_collection,
                                                filter_metadata=filter_metadata,
                                                search_type=search_type)
                if results:
                    self.resource_manager.ensure_vram(self.reranker.vram_required)
                    results = self.reranker.rerank(query_text, results, top_k=final_top_k)
                    reranked = True
            else:
                results = self.retriever.search(query_embedding, top_k=final_top_k,
                                                collection_name=resolved_collection,
                                                filter_metadata=filter_metadata,
                                                search_type=search_type)

            if not results:
                return QueryResult(query=query_text, collection_name=resolved_collection,
                                   results=[], reranked=reranked, search_type=search_type,
                                   hyde_used=hyde_used, expanded_query=expanded_query)

            response_text = self._build_response(query_text, results)
            generated_answer = None
            if generate_answer and self.generator is not None:
                try:
                    generated_answer = self.generator.generate(query_text, results)
                except Exception as e:
                    logger.warning(f"Generation failed: {e}")
            audio_path = None
            if generate_audio:
                raise NotImplementedError("TTS is not part of the MI355X build")
            return QueryResult(query=query_text, collection_name=resolved_collection,
                               results=results, response_text=response_text,
                               generated_answer=generated_answer, audio_path=audio_path,
                               reranked=reranked, search_type=search_type, hyde_used=hyde_used,
                               expanded_query=expanded_query)
        except Exception as e:
            logger.error(f"Query failed: {e}")
            raise PipelineError(f"Query failed: {e}") from e

    def _build_response(self, query: str, results: list[RetrievalResult]) -> str:
        """query.py:217-226."""
        if not results:
            return "No relevant information found."
        parts = []
        for result in results:
            chunk = result.chunk
            speaker = chunk.speaker or "Unknown"
            time_str = f"{chunk.start:.1f}s-{chunk.end:.1f}s"
            parts.append(f"[{speaker} at {time_str}]: {chunk.text}")
        return "\n\n".join(parts)

    def get_context_for_llm(self, query: str, collection_name: str | None = None,
                            top_k: int | None = None, filter_metadata: dict | None = None) -> str:
        """query.py:228-255."""
        resolved_collection = collection_name or self.config.retrieval.collection_name
        try:
            self.resource_manager.ensure_vram(self.embedder.vram_required)
            query_embedding = self.embedder.embed_query(query)
            results = self.retriever.search(query_embedding, top_k=top_k,
                                            collection_name=resolved_collection,
                                            filter_metadata=filter_metadata)
            if not results:
                return "No relevant context found."
            parts = []
            for result in results:
                chunk = result.chunk
                speaker = chunk.speaker or "Speaker"
                source = chunk.metadata.get("source_filename", "unknown") if chunk.metadata else "unknown"
                parts.append(f"<context speaker=\"{speaker}\" start=\"{chunk.start:.1f}\" "
                             f"end=\"{chunk.end:.1f}\" source=\"{source}\" score=\"{result.score:.3f}\">\n"
                             f"{chunk.text}\n</context>")
            return "\n\n".join(parts)
        except Exception as e:
            raise PipelineError(f"Failed to get context: {e}") from e

    # --------------------------------------------------------------------- batched path

    def query_batch(self, query_texts: list[str], collection_name: str | None = None,
                    top_k: int | None = None, filter_metadata: dict | None = None,
                    search_type: str | None = None, enable_reranking: bool = True) -> list[QueryResult]:
        """Per-query semantics of query() (no HyDE / generation / TTS), executed as device
        batches: one encoder pass, one retrieval pass (dense / sparse / RRF kernels over all
        queries), one cross-encoder pass over every (query, candidate) pair."""
        resolved = collection_name or self.config.retrieval.collection_name
        final_top_k = top_k or self.config.reranking.top_k
        search_type = search_type or self.config.retrieval.search_type
        try:
            retriever = self.retriever
            dense, lex = self.embedder.embed_queries(query_texts)
            use_rerank = enable_reranking and self.reranker is not None
            k = self.config.reranking.initial_k if use_rerank else final_top_k
            # query() searches a query without lexical weights (_convert_sparse -> None) dense
            # and the others with their sparse vector: one device batch per such group
            has_lex = [bool(x) for x in lex] if lex is not None else [False] * len(query_texts)
            per_query: list = [None] * len(query_texts)
            # a sharded retriever's search_batch is a collective (one all-gather per call): every
            # rank must make the same number of calls whatever its own queries are, so both groups
            # are searched even when one is empty (search_batch takes an empty batch)
            collective = getattr(retriever, "_world", 1) > 1
            for want in (True, False):
                rows = [i for i, h in enumerate(has_lex) if h == want]
                if not rows and not collective:
                    continue
                sel = torch.tensor(rows, dtype=torch.long, device=dense.device)
                batch = QueryBatch(dense=dense.index_select(0, sel).contiguous())
                if want:
                    parts = [query_sparse_arrays(self.embedder._convert_sparse(lex[i])) for i in rows]
                    indptr = np.zeros(len(parts) + 1, dtype=np.int32)
                    np.cumsum([len(p[0]) for p in parts], out=indptr[1:])
                    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(retriever.device)
                    # one unused entry keeps the term arrays non-empty (an empty group, or queries
                    # whose terms were all dropped): the C ABI refuses null arrays
                    batch = QueryBatch(dense=batch.dense, sparse_indptr=t(indptr),
                                       sparse_indices=t(np.concatenate([p[0] for p in parts] +
                                                                       [np.zeros(1, np.int32)])),
                                       sparse_values=t(np.concatenate([p[1] for p in parts] +
                                                                      [np.zeros(1, np.float32)])))
                out, mode = retriever.search_batch(batch, k, resolved, filter_metadata, search_type)
                thr = None  # search()'s score_threshold rule (qdrant.py:331: legacy dense only)
                if mode == "legacy_dense" and self.config.retrieval.score_threshold > 0:
                    thr = self.config.retrieval.score_threshold
                for b, i in enumerate(rows):
                    per_query[i] = retriever.materialize(out, mode, resolved, b, thr)
            results = []
            if use_rerank:
                per_query = self._rerank_batch(query_texts, per_query, final_top_k)
            for q, res in zip(query_texts, per_query):
                results.append(QueryResult(query=q, collection_name=resolved, results=res,
                                           response_text=self._build_response(q, res) if res else None,
                                           reranked=use_rerank and bool(res), search_type=search_type))
            return results
        except Exception as e:
            raise PipelineError(f"Query failed: {e}") from e

    def _rerank_batch(self, queries: list[str], per_query: list[list[RetrievalResult]],
                      top_k: int) -> list[list[RetrievalResult]]:
        """BGEReranker.rerank rules per query, with all model calls in one device batch."""
        rr = self.reranker
        todo = [i for i, res in enumerate(per_query) if len(res) > top_k]
        out = [sorted(res, key=lambda x: x.score, reverse=True) if len(res) <= top_k else None
               for res in per_query]
        if todo:
            try:
                from audio_rag_amd.text import pair_ids

                pairs, owner = [], []
                for i in todo:
                    q = rr.tokenizer.tokenize(queries[i])
                    for r in per_query[i]:
                        pairs.append(pair_ids(q, rr.tokenizer.tokenize(r.chunk.text), rr.config.max_length))
                        owner.append(i)
                scores = rr.score_ids(pairs).cpu().tolist()
                pos = 0
                for i in todo:
                    n = len(per_query[i])
                    new = [RetrievalResult(chunk=r.chunk, score=float(scores[pos + j]))
                           for j, r in enumerate(per_query[i])]
                    pos += n
                    new.sort(key=lambda x: x.score, reverse=True)
                    out[i] = new[:top_k]
            except Exception as e:
                logger.warning(f"Reranking failed: {e}, returning original top-{top_k}")
                for i in todo:
                    out[i] = sorted(per_query[i], key=lambda x: x.score, reverse=True)[:top_k]
        return out

    def unload_all(self) -> None:
        if self._embedder and self._embedder.is_loaded:
            self._embedder.unload()
        if self._reranker and self._reranker.is_loaded:
            self._reranker.unload()
