"""Generic component registry (same contract as src/audio_rag/core/registry.py:8-58).

A duplicate key raises ValueError (registry.py:30-31); an unknown key raises KeyError listing
what is available (registry.py:36-41).
"""

from typing import Any, Callable, Generic, TypeVar

T = TypeVar("T")


class Registry(Generic[T]):
    def __init__(self, name: str):
        self.name = name
        self._registry: dict[str, type[T]] = {}

    def register(self, key: str) -> Callable[[type[T]], type[T]]:
        def decorator(cls: type[T]) -> type[T]:
            if key in self._registry:
                raise ValueError(f"{self.name}: '{key}' already registered")
            self._registry[key] = cls
            return cls

        return decorator

    def _missing(self, key: str) -> KeyError:
        available = ", ".join(self._registry.keys()) or "none"
        return KeyError(f"{self.name}: '{key}' not found. Available: {available}")

    def create(self, key: str, **kwargs: Any) -> T:
        if key not in self._registry:
            raise self._missing(key)
        return self._registry[key](**kwargs)

    def get(self, key: str) -> type[T]:
        if key not in self._registry:
            raise self._missing(key)
        return self._registry[key]

    def list(self) -> list[str]:
        return list(self._registry.keys())

    def __contains__(self, key: str) -> bool:
        return key in self._registry

    def __repr__(self) -> str:
        return f"Registry({self.name}, components={self.list()})"
