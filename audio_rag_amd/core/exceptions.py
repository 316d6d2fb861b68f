"""Exception hierarchy of the query path (mirrors src/audio_rag/core/exceptions.py:1-66)."""


class AudioRAGError(Exception):
    """Base exception for all Audio RAG errors."""


class ConfigError(AudioRAGError):
    """Configuration loading or validation error."""


class RegistryError(AudioRAGError):
    """Component registry error."""


class ResourceError(AudioRAGError):
    """Resource management error (VRAM, memory, etc.)."""


class EmbeddingError(AudioRAGError):
    """Embedding generation error."""


class RetrievalError(AudioRAGError):
    """Vector retrieval error."""


class PipelineError(AudioRAGError):
    """Pipeline orchestration error."""


class GenerationError(AudioRAGError):
    """LLM answer generation error."""


class RerankingError(AudioRAGError):
    """Reranking error."""
