"""Retrieval registry (mirrors src/audio_rag/retrieval/base.py:6)."""

from audio_rag_amd.core import BaseRetriever, Registry

RetrievalRegistry = Registry[BaseRetriever]("retrieval")
