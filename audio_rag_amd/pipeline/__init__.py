"""Query pipeline and facade (mirrors src/audio_rag/pipeline/__init__.py, query side)."""

from audio_rag_amd.pipeline.orchestrator import AudioRAG
from audio_rag_amd.pipeline.query import QueryPipeline, QueryResult

__all__ = ["AudioRAG", "QueryPipeline", "QueryResult"]
