"""Sparse top-k micro-benchmark: the bench.py synthetic corpus (1M rows, ~96 postings per row,
Zipf(1.1) ids) and 64-query batches, timed with events on the launch stream.

python tools/sparse_bench.py [--rows N] [--batches B] [--iters I]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from audio_rag_amd.retrieval.device import SparseIndex  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--filter", choices=["on", "off"], default="on",
                    help="armi_sparse_topk's MFMA filter (off: the exact scan alone)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    t0 = time.time()
    indptr, idx, val = bench.make_sparse_rows(0, a.rows, dev)
    torch.cuda.synchronize()
    t1 = time.time()
    si = SparseIndex(indptr, idx, val, bench.VOCAB)
    si.set_filter(a.filter == "on")
    torch.cuda.synchronize()
    t2 = time.time()
    print(f"corpus {a.rows} rows nnz {idx.numel()} gen {t1 - t0:.2f}s build {t2 - t1:.3f}s", flush=True)
    qs = [bench.make_sparse_queries(a.batch, dev, seed=100 + i) for i in range(4)]
    ws = torch.empty(si.workspace_bytes(a.batch, a.k), dtype=torch.uint8, device=dev)
    for q in qs:
        si.topk(*q, a.k, workspace=ws)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for i in range(a.iters):
        r = si.topk(*qs[i % len(qs)], a.k, workspace=ws)
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / a.iters
    fl = r.flags.cpu()
    print(f"batch {a.batch} k {a.k}: {ms:.3f} ms/batch, {a.batch / ms * 1e3:.0f} queries/s, "
          f"certified {(fl & 1).bool().float().mean().item():.2f} "
          f"filtered {(fl & 4).bool().float().mean().item():.2f} (filter {a.filter})", flush=True)


if __name__ == "__main__":
    main()
