"""Reranking (mirrors src/audio_rag/reranking/__init__.py)."""

from audio_rag_amd.reranking.base import BaseReranker, RerankerRegistry
from audio_rag_amd.reranking.bge import BGEReranker

__all__ = ["BaseReranker", "RerankerRegistry", "BGEReranker"]
