"""Reranker ABC and registry (mirrors src/audio_rag/reranking/base.py:13-84).

RerankerRegistry.create("none") returns None (base.py:74-76), which makes QueryPipeline skip
reranking."""

from abc import ABC, abstractmethod

from audio_rag_amd.config.schema import RerankingConfig
from audio_rag_amd.core.base import RetrievalResult


class BaseReranker(ABC):
    def __init__(self, config: RerankingConfig):
        self.config = config
        self._is_loaded = False

    @property
    def is_loaded(self) -> bool:
        return self._is_loaded

    @property
    @abstractmethod
    def vram_required(self) -> float: ...

    @abstractmethod
    def load(self) -> None: ...

    @abstractmethod
    def unload(self) -> None: ...

    @abstractmethod
    def rerank(self, query: str, results: list[RetrievalResult],
               top_k: int | None = None) -> list[RetrievalResult]: ...


class RerankerRegistry:
    _rerankers: dict[str, type[BaseReranker]] = {}

    @classmethod
    def register(cls, name: str):
        def decorator(reranker_cls):
            cls._rerankers[name] = reranker_cls
            return reranker_cls

        return decorator

    @classmethod
    def create(cls, name: str, config: RerankingConfig) -> BaseReranker | None:
        if name == "none":
            return None
        if name not in cls._rerankers:
            raise ValueError(f"Unknown reranker: {name}. Available: {list(cls._rerankers)}")
        return cls._rerankers[name](config)

    @classmethod
    def list_available(cls) -> list[str]:
        return list(cls._rerankers.keys())
