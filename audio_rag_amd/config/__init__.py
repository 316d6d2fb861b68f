from audio_rag_amd.config.loader import load_config
from audio_rag_amd.config.schema import (AudioRAGConfig, EmbeddingConfig, ExpansionConfig,
                                         GenerationConfig, RerankingConfig, RetrievalConfig)

__all__ = ["AudioRAGConfig", "EmbeddingConfig", "RetrievalConfig", "RerankingConfig",
           "ExpansionConfig", "GenerationConfig", "load_config"]
