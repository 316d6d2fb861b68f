"""AudioRAG facade, query side (mirrors src/audio_rag/pipeline/orchestrator.py:16-193).

The lazy wiring is the reference's: the first access to .retriever loads the embedder (to learn
the dimension) and creates the retriever from the registry (orchestrator.py:48-57); the query
pipeline shares the facade's embedder and retriever (68-75). Audio ingestion (ASR, diarization,
chunking) is out of scope; add_chunks() is the ingest entry for pre-chunked text and
pre-computed embeddings (the embed + add tail of IngestionPipeline.ingest, ingestion.py:176-185).
"""

from __future__ import annotations

from pathlib import Path

from audio_rag_amd.config import AudioRAGConfig, load_config
from audio_rag_amd.core.base import AudioChunk, EmbeddingResult
from audio_rag_amd.embeddings import EmbeddingsRegistry
from audio_rag_amd.pipeline.components import ResourceManager
from audio_rag_amd.pipeline.query import QueryPipeline, QueryResult
from audio_rag_amd.retrieval import RetrievalRegistry
from audio_rag_amd.utils import setup_logging


class AudioRAG:
    def __init__(self, config: AudioRAGConfig):
        self.config = config
        setup_logging(level=config.log_level)
        self.resource_manager = ResourceManager(config.resources)
        self._embedder = None
        self._retriever = None
        self._query_pipeline = None

    @classmethod
    def from_config(cls, config_path: Path | str | None = None, env: str | None = None,
                    config_dir: Path | str = "configs") -> "AudioRAG":
        return cls(load_config(config_path=config_path, env=env, config_dir=config_dir))

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
    def query_pipeline(self) -> QueryPipeline:
        if self._query_pipeline is None:
            self._query_pipeline = QueryPipeline(config=self.config,
                                                 resource_manager=self.resource_manager)
            self._query_pipeline._embedder = self.embedder
            self._query_pipeline._retriever = self.retriever
        return self._query_pipeline

    def add_chunks(self, chunks: list[AudioChunk], embeddings: list[EmbeddingResult] | None = None,
                   collection_name: str | None = None) -> int:
        if embeddings is None:
            embeddings = self.embedder.embed([c.text for c in chunks])
        self.retriever.add(chunks, embeddings, collection_name=collection_name)
        return len(chunks)

    def query(self, query_text: str, collection_name: str | None = None, top_k: int | None = None,
              filter_metadata: dict | None = None, search_type: str | None = None,
              enable_hyde: bool | None = None, enable_reranking: bool = True,
              generate_answer: bool = True, generate_audio: bool = False,
              audio_output_path: Path | str | None = None) -> QueryResult:
        return self.query_pipeline.query(
            query_text=query_text, collection_name=collection_name, top_k=top_k,
            filter_metadata=filter_metadata, search_type=search_type, enable_hyde=enable_hyde,
            enable_reranking=enable_reranking, generate_answer=generate_answer,
            generate_audio=generate_audio, audio_output_path=audio_output_path)

    def query_batch(self, query_texts: list[str], **kwargs) -> list[QueryResult]:
        return self.query_pipeline.query_batch(query_texts, **kwargs)

    def get_context(self, query: str, collection_name: str | None = None, top_k: int | None = None,
                    filter_metadata: dict | None = None) -> str:
        return self.query_pipeline.get_context_for_llm(query=query, collection_name=collection_name,
                                                       top_k=top_k, filter_metadata=filter_metadata)

    def status(self) -> dict:
        return {
            "config": {
                "embedding_backend": self.config.embedding.backend,
                "embedding_sparse": self.config.embedding.use_sparse,
                "retrieval_backend": self.config.retrieval.backend,
                "retrieval_search_type": self.config.retrieval.search_type,
                "reranking_backend": self.config.reranking.backend,
                "expansion_backend": self.config.expansion.backend,
                "generation_backend": self.config.generation.backend,
            },
            "resources": self.resource_manager.status(),
            "collection": {
                "name": self.config.retrieval.collection_name,
                "count": self.retriever.count() if self._retriever else 0,
            },
        }

    def clear_collection(self, collection_name: str | None = None) -> None:
        self.retriever.delete_collection(collection_name)

    def unload_all(self) -> None:
        if self._query_pipeline:
            self._query_pipeline.unload_all()
        if self._embedder and self._embedder.is_loaded:
            self._embedder.unload()
