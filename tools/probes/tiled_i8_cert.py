"""Certified fraction and call time of the dense top-5 over (rows, queries) shapes (one GPU):
the tiled scans of the sharded step's all-gathered batch."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from audio_rag_amd.retrieval.device import DenseIndex  # noqa: E402
from audio_rag_amd.synthetic import make_queries, make_rows  # noqa: E402

dev = torch.device("cuda", 0)
shapes = [(20_000, 512), (65_536, 512), (125_000, 512), (250_000, 256), (500_000, 512),
          (1_000_000, 256), (1_250_000, 512)]
for n, b in shapes:
    rows = make_rows(0, n, 1024, dev)
    idx = DenseIndex(rows)
    q = make_queries(1, b, 1024, dev, seed=1)[0]
    ws = torch.empty(idx.workspace_bytes(b, 5), dtype=torch.uint8, device=dev)
    for _ in range(3):
        out = idx.topk(q, 5, workspace=ws)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        out = idx.topk(q, 5, workspace=ws)
    e1.record()
    torch.cuda.synchronize()
    f = out.flags.cpu()
    print(f"rows {n} queries {b} form {idx.scan_form(b, 5)} certified "
          f"{f.eq(1).float().mean().item():.4f} call {e0.elapsed_time(e1) / 10 * 1e3:.1f} us",
          flush=True)
    idx.close()
    del rows, ws
    torch.cuda.empty_cache()
