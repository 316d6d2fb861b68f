"""Embeddings registry (mirrors src/audio_rag/embeddings/base.py:6)."""

from audio_rag_amd.core import BaseEmbedder, Registry

EmbeddingsRegistry = Registry[BaseEmbedder]("embeddings")
