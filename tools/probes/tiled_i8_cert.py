"""Certified fraction of the int8 tiled scan over (rows, queries) shapes (one GPU)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from audio_rag_amd import _armi  # noqa: E402
from audio_rag_amd.retrieval.device import DenseIndex  # noqa: E402
from audio_rag_amd.synthetic import make_queries, make_rows  # noqa: E402

dev = torch.device("cuda", 0)
for n, b in [(1_000_000, 256), (1_000_000, 300), (1_250_000, 256), (1_250_000, 512), (600_000, 256),
             (1_000_000, 512)]:
    rows = make_rows(0, n, 1024, dev)
    idx = DenseIndex(rows)
    q = make_queries(1, b, 1024, dev, seed=1)[0]
    out = idx.topk(q, 5)
    torch.cuda.synchronize()
    f = out.flags.cpu()
    print(n, b, "form", idx.scan_form(b, 5), "certified", f.eq(1).float().mean().item(),
          "flags", torch.unique(f, return_counts=True), flush=True)
    idx.close()
    del rows
    torch.cuda.empty_cache()
