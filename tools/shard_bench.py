"""Per-GPU compute of the sharded bench step, emulated on one GPU: armi_dense_topk of G*64
queries over a 1/G shard of the 1M-row corpus (what every rank runs between the two
all-gathers at N = G), timed with HIP events. Prints one line per G.

    python tools/shard_bench.py [--iters 20] [--k 5]
"""

import argparse
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--k", type=int, default=5)
    ap.add_argument("--chunks", type=int, default=1_000_000)
    ap.add_argument("--gs", default="1,2,4,8")
    args = ap.parse_args()
    from bench import make_queries, make_rows
    from audio_rag_amd import _armi
    from audio_rag_amd.retrieval.device import DenseIndex

    dev = torch.device("cuda", 0)
    for g in (int(x) for x in args.gs.split(",")):
        n = args.chunks // g
        rows = make_rows(0, n, 1024, dev)
        idx = DenseIndex(rows)
        q = make_queries(1, 64 * g, 1024, dev, seed=1)[0]
        ws = torch.empty(idx.workspace_bytes(64 * g, args.k), dtype=torch.uint8, device=dev)
        for _ in range(3):
            out = idx.topk(q, args.k, workspace=ws)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        tot = _armi.ctypes.c_double()
        launches = _armi.ctypes.c_int64()
        _armi.call("armi_scan_timing_enable", 1)
        _armi.call("armi_scan_timing_read", _armi.ctypes.byref(tot), _armi.ctypes.byref(launches))
        a.record()
        for _ in range(args.iters):
            out = idx.topk(q, args.k, workspace=ws)
        b.record()
        torch.cuda.synchronize()
        _armi.call("armi_scan_timing_read", _armi.ctypes.byref(tot), _armi.ctypes.byref(launches))
        _armi.call("armi_scan_timing_enable", 0)
        ms = a.elapsed_time(b) / args.iters
        scan_ms = tot.value / max(launches.value, 1)
        tflops = 2.0 * n * 1024 * 64 * g / (scan_ms * 1e-3) / 1e12
        cert = float((out.flags == 1).float().mean().item())
        print(f"G={g} shard_rows={n} queries={64 * g} k={args.k}: {ms * 1e3:.1f} us per call, "
              f"{64 * g / (ms * 1e-3):.0f} q/s per GPU, certified {cert:.3f}; scan kernel "
              f"{scan_ms * 1e3:.1f} us ({tflops:.0f} TFLOP/s)", flush=True)
        del idx, rows, ws


if __name__ == "__main__":
    main()
