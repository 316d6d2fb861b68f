"""audio_rag_amd — MI355X-native query-time retrieval hot path of audio-rag.

Drop-in for the reference's AudioRAG.query() / retriever.search() surface
(src/audio_rag/pipeline/orchestrator.py:117-140, src/audio_rag/retrieval/qdrant.py:227-352):
dense cosine top-k, sparse lexical top-k, RRF fusion and the cross-encoder's non-GEMM ops run as
hand-written HIP kernels for gfx950 behind the C ABI of include/armi.h (libarmi.so).
"""

__version__ = "0.1.0"

__all__ = ["AudioRAG", "QueryPipeline", "QueryResult", "AudioRAGConfig", "load_config"]


def __getattr__(name):  # lazy: importing the package must not initialise the GPU
    if name in ("AudioRAG",):
        from audio_rag_amd.pipeline.orchestrator import AudioRAG
        return AudioRAG
    if name in ("QueryPipeline", "QueryResult"):
        from audio_rag_amd.pipeline import query as _q
        return getattr(_q, name)
    if name in ("AudioRAGConfig", "load_config"):
        from audio_rag_amd import config as _c
        return getattr(_c, name)
    raise AttributeError(name)
