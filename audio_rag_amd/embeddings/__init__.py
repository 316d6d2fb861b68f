"""Embedding backends (mirrors src/audio_rag/embeddings/__init__.py)."""

from audio_rag_amd.embeddings.base import EmbeddingsRegistry
from audio_rag_amd.embeddings.bge_m3 import BGEM3Embedder

__all__ = ["EmbeddingsRegistry", "BGEM3Embedder"]
