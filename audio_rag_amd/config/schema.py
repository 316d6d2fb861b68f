"""Pydantic configuration of the query path.

The sections and defaults the hot path reads are those of src/audio_rag/config/schema.py:48-133
(EmbeddingConfig 48-55, RetrievalConfig 58-69, RerankingConfig 72-79, ExpansionConfig 82-85,
GenerationConfig 88-96). Differences, all additive:
  * RetrievalConfig.backend accepts "mi355x" (the device chunk store of this package) and
    defaults to it. "qdrant" (what the reference's configs/base.yaml:39 names) resolves to the
    same MI355X store, so reference config files build a working pipeline unchanged; the Qdrant
    connection knobs (qdrant_host / qdrant_port / qdrant_in_memory) are accepted and ignored.
  * RetrievalConfig.device / rrf_k / reproduce_sparse_drop and RerankingConfig.max_length are new
    knobs of the MI355X backend (rrf_k = 2 is Qdrant's RRF constant, 1/(rrf_k + pos)).
  * reproduce_sparse_drop defaults to True: add() then stores what the reference's add() leaves
    in Qdrant (qdrant.py:183-220 upserts dense+sparse points, then re-upserts the same ids
    dense-only, which replaces them), so a hybrid search over a corpus ingested through add()
    returns the reference's results. False keeps the sparse vectors (an explicit opt-in bug
    fix, not the reference's behaviour).
Sections of the ingestion side (asr, diarization, alignment, chunking, contextual, tts,
resources) are accepted as free-form dicts so reference YAML files load unchanged.
"""

from typing import Any, Literal

from pydantic import BaseModel, Field


class EmbeddingConfig(BaseModel):
    backend: Literal["bge-m3", "multilingual-e5"] = "bge-m3"
    model: str = "BAAI/bge-m3"
    device: Literal["cuda", "cpu", "auto"] = "auto"
    batch_size: int = Field(default=32, ge=1)
    normalize: bool = True
    use_sparse: bool = True
    # MI355X build: weights are not on disk; the encoder is initialised from this seed
    seed: int = 0
    max_length: int = Field(default=8192, ge=8)
    # batch-1 query encodes replay a HIP graph captured per padded length bucket (16, 32, 64,
    # ..., 512 tokens) instead of re-launching the 24-layer forward kernel by kernel
    query_graphs: bool = True


class RetrievalConfig(BaseModel):
    backend: Literal["qdrant", "mi355x"] = "mi355x"
    collection_name: str = "audio_rag"
    search_type: Literal["dense", "sparse", "hybrid"] = "hybrid"
    top_k: int = Field(default=5, ge=1, le=100)
    score_threshold: float = Field(default=0.0, ge=0.0, le=1.0)
    qdrant_host: str = "localhost"
    qdrant_port: int = 6333
    qdrant_in_memory: bool = False
    dense_weight: float = Field(default=0.7, ge=0.0, le=1.0)   # never read (as in the reference)
    sparse_weight: float = Field(default=0.3, ge=0.0, le=1.0)  # never read (as in the reference)
    # MI355X backend
    device: int = 0
    rrf_k: int = Field(default=2, ge=1)
    reproduce_sparse_drop: bool = True
    # unfiltered single-query search() replays a HIP graph captured per (collection, branch,
    # top_k): one host->device copy of the query, one replay of the search kernels, one
    # device->host copy of the packed result
    query_graphs: bool = True
    # GPUs the corpus is sharded over: > 1 runs one process per GPU
    # (torchrun), torch.distributed initialised before the retriever; searches are collective
    # calls (MI355XRetriever._search_sharded)
    num_gpus: int = Field(default=1, ge=1)


class RerankingConfig(BaseModel):
    backend: Literal["bge-reranker", "none"] = "bge-reranker"
    model: str = "BAAI/bge-reranker-base"
    device: Literal["cuda", "cpu", "auto"] = "auto"
    top_k: int = Field(default=5, ge=1, le=50)
    initial_k: int = Field(default=20, ge=1, le=100)
    batch_size: int = Field(default=16, ge=1)
    # MI355X build
    seed: int = 5
    max_length: int = Field(default=512, ge=8, le=512)
    # cross-encoder compute: "fp16" = fp16 GEMMs + fused fp16 attention (scores within 1e-4 of
    # the fp32 forward, north_star budget 1e-3); "fp32" = sentence-transformers' default dtype
    dtype: Literal["fp16", "fp32"] = "fp16"


class ExpansionConfig(BaseModel):
    backend: Literal["hyde", "none"] = "none"
    num_hypotheses: int = Field(default=1, ge=1, le=3)


class GenerationConfig(BaseModel):
    backend: Literal["ollama", "none"] = "ollama"
    model: str = "llama3.2:3b"
    base_url: str = "http://localhost:11434"
    temperature: float = Field(default=0.7, ge=0.0, le=2.0)
    max_tokens: int = Field(default=1024, ge=1, le=8192)
    timeout: float = Field(default=60.0, ge=1.0)
    fallback_models: list[str] = Field(default_factory=lambda: ["llama3.1:8b", "mistral:7b"])


class AudioRAGConfig(BaseModel):
    embedding: EmbeddingConfig = Field(default_factory=EmbeddingConfig)
    retrieval: RetrievalConfig = Field(default_factory=RetrievalConfig)
    reranking: RerankingConfig = Field(default_factory=RerankingConfig)
    expansion: ExpansionConfig = Field(default_factory=ExpansionConfig)
    generation: GenerationConfig = Field(default_factory=GenerationConfig)
    # ingestion-side sections: accepted, not interpreted by the query path
    asr: dict[str, Any] = Field(default_factory=dict)
    diarization: dict[str, Any] = Field(default_factory=dict)
    alignment: dict[str, Any] = Field(default_factory=dict)
    chunking: dict[str, Any] = Field(default_factory=dict)
    contextual: dict[str, Any] = Field(default_factory=dict)
    tts: dict[str, Any] = Field(default_factory=dict)
    resources: dict[str, Any] = Field(default_factory=dict)
    log_level: Literal["DEBUG", "INFO", "WARNING", "ERROR"] = "INFO"
    data_dir: str = "./data"
    cache_dir: str = "./cache"
