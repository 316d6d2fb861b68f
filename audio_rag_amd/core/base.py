"""Boundary types and plugin ABCs of the query path.

Field-for-field the dataclasses of src/audio_rag/core/base.py:29-61 (AudioChunk, SparseVector,
EmbeddingResult, RetrievalResult) and the embedder / retriever ABCs of base.py:128-190, so
results built here are interchangeable with the reference's.
"""

from abc import ABC, abstractmethod
from dataclasses import dataclass


@dataclass
class AudioChunk:
    """A chunk of audio transcript ready for embedding (core/base.py:29-36)."""

    text: str
    start: float
    end: float
    speaker: str | None = None
    metadata: dict | None = None


@dataclass
class SparseVector:
    """Sparse lexical-weight vector (core/base.py:39-46)."""

    indices: list[int]
    values: list[float]

    def to_dict(self) -> dict[int, float]:
        return dict(zip(self.indices, self.values))


@dataclass
class EmbeddingResult:
    """Dense and optional sparse embedding (core/base.py:49-53)."""

    dense: list[float]
    sparse: SparseVector | None = None


@dataclass
class RetrievalResult:
    """A retrieved chunk with relevance score (core/base.py:56-61)."""

    chunk: AudioChunk
    score: float
    source: str | None = None


class BaseEmbedder(ABC):
    """core/base.py:128-167."""

    @abstractmethod
    def embed(self, texts: list[str]) -> list[EmbeddingResult]: ...

    @abstractmethod
    def embed_query(self, query: str) -> EmbeddingResult: ...

    @abstractmethod
    def load(self) -> None: ...

    @abstractmethod
    def unload(self) -> None: ...

    @property
    @abstractmethod
    def is_loaded(self) -> bool: ...

    @property
    @abstractmethod
    def vram_required(self) -> float: ...

    @property
    @abstractmethod
    def dimension(self) -> int: ...

    @property
    def supports_sparse(self) -> bool:
        return False


class BaseRetriever(ABC):
    """core/base.py:170-190. Live callers also pass search_type= (pipeline/query.py:152,167)."""

    @abstractmethod
    def add(self, chunks: list[AudioChunk], embeddings: list[EmbeddingResult],
            collection_name: str | None = None) -> None: ...

    @abstractmethod
    def search(self, query_embedding: EmbeddingResult, top_k: int | None = None,
               collection_name: str | None = None,
               filter_metadata: dict | None = None) -> list[RetrievalResult]: ...
