"""Core boundary types, registry and exceptions (mirrors src/audio_rag/core/__init__.py)."""

from audio_rag_amd.core.base import (AudioChunk, BaseEmbedder, BaseRetriever, EmbeddingResult,
                                     RetrievalResult, SparseVector)
from audio_rag_amd.core.exceptions import (AudioRAGError, ConfigError, EmbeddingError,
                                           GenerationError, PipelineError, RegistryError,
                                           RerankingError, ResourceError, RetrievalError)
from audio_rag_amd.core.registry import Registry

__all__ = [
    "AudioChunk", "SparseVector", "EmbeddingResult", "RetrievalResult", "BaseEmbedder",
    "BaseRetriever", "Registry", "AudioRAGError", "ConfigError", "RegistryError", "ResourceError",
    "EmbeddingError", "RetrievalError", "PipelineError", "GenerationError", "RerankingError",
]
