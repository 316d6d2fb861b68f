"""Retrieval backends (mirrors src/audio_rag/retrieval/__init__.py).

"mi355x" is this package's device chunk store; importing the module registers it.
"""

from audio_rag_amd.retrieval.base import RetrievalRegistry
from audio_rag_amd.retrieval.mi355x import MI355XRetriever

__all__ = ["RetrievalRegistry", "MI355XRetriever"]
