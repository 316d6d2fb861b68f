"""Batch-1 BGE-M3 query encode (captured graph on the armi encoder kernels) for rocprofv3:
per-kernel durations of the 24-layer forward."""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from audio_rag_amd.config import EmbeddingConfig  # noqa: E402
from audio_rag_amd.embeddings.bge_m3 import BGEM3Embedder  # noqa: E402

dev = torch.device("cuda", 0)
e = BGEM3Embedder(EmbeddingConfig(), device=dev)
e.load()
seq = e.tokenizer.encode("what does the lecturer say about gradient descent")
for _ in range(5):
    e.encode_query_ids(seq)
torch.cuda.synchronize()
t = []
for _ in range(50):
    t0 = time.perf_counter()
    e.encode_query_ids(seq)
    torch.cuda.synchronize()
    t.append(time.perf_counter() - t0)
t.sort()
print(f"L={len(seq)} p50 {t[len(t) // 2] * 1e3:.3f} ms")
