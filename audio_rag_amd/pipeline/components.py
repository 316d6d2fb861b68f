"""Stand-ins for the query path's out-of-scope neighbours, keeping the
reference's observable behaviour when those services are unreachable:

  * HyDE expansion (expansion/hyde.py, Ollama over HTTP): is_available is False, so
    QueryPipeline embeds the original query (query.py:127-134 skip when unavailable).
  * Answer generation (generation/ollama.py): generate() raises GenerationError, which
    QueryPipeline logs as a warning and leaves generated_answer None (query.py:185-190).
  * TTS (tts/): not part of this build; generate_audio=True raises inside the pipeline's try
    and surfaces as PipelineError like any other failure (query.py:213-215).
  * ResourceManager.ensure_vram (resources/manager.py:106-153): a no-op in the reference
    because no model is ever registered (manager.py:71-97); kept as a no-op.
"""

from __future__ import annotations

from audio_rag_amd.core.exceptions import GenerationError


class HyDEExpander:
    def __init__(self, config=None):
        self.config = config

    @property
    def is_available(self) -> bool:
        return False

    def expand_single(self, query: str) -> str:
        return query


class OllamaGenerator:
    def __init__(self, config=None):
        self.config = config

    def generate(self, query: str, results) -> str:
        raise GenerationError("answer generation (Ollama) is not part of the MI355X build")


class GeneratorRegistry:
    @staticmethod
    def create(name: str, config=None):
        if name == "none":
            return None
        if name == "ollama":
            return OllamaGenerator(config)
        raise ValueError(f"Unknown generator: {name}")


class ResourceManager:
    def __init__(self, config=None):
        self.config = config

    def ensure_vram(self, required_gb: float) -> bool:
        return True

    def status(self) -> dict:
        return {"registered_models": 0}

    def unload_all(self) -> None:
        pass
