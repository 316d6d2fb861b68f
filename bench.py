"""Benchmark of the MI355X retrieval hot path (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json metric "queries/sec + p50 latency, 1M x 1024-d chunks, top-5"):
  a 1M x 1024 fp16 chunk store (synthetic unit vectors) sharded by chunk
  ordinal over the N GPUs; every step each GPU brings its own batch of 64 queries; a step is
    all-gather queries (RCCL) -> armi_dense_topk of all N*64 queries on the local shard ->
    all-gather the per-shard top-5 (RCCL) -> armi_topk_merge_shards of this GPU's 64 queries.
  At N=1 the collectives vanish. Per-GPU work is fixed (shard rows x N*64 queries = 1M x 64),
  so scaling is weak; value = all queries answered by all GPUs / time.
Inputs are resident in HBM before the timed region; the timed region is K steps bracketed by a
barrier + synchronize on both sides, max over ranks.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = json.loads((ROOT / "BASELINE.json").read_text())["metric"]
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
CHUNK_ROWS = 65536


def make_rows(first: int, count: int, dim: int, device, seed: int = 0) -> torch.Tensor:
    """Rows [first, first+count) of the global synthetic corpus: each 64k-row chunk has its own
    seed, so a shard's rows are identical whatever the shard count."""
    out = torch.empty((count, dim), dtype=torch.float16, device=device)
    c0 = first // CHUNK_ROWS
    c1 = (first + count + CHUNK_ROWS - 1) // CHUNK_ROWS
    for c in range(c0, c1):
        a, b = c * CHUNK_ROWS, (c + 1) * CHUNK_ROWS
        g = torch.Generator(device=device).manual_seed(seed * 1_000_003 + c)
        x = torch.randn((CHUNK_ROWS, dim), generator=g, device=device)
        x = (x / x.norm(dim=1, keepdim=True)).half()
        lo, hi = max(a, first), min(b, first + count)
        if lo < hi:
            out[lo - first:hi - first] = x[lo - a:hi - a]
    return out


def make_queries(n_batches: int, batch: int, dim: int, device, seed: int) -> torch.Tensor:
    g = torch.Generator(device=device).manual_seed(seed)
    x = torch.randn((n_batches, batch, dim), generator=g, device=device)
    return (x / x.norm(dim=2, keepdim=True)).half().contiguous()


def cpu_baseline(n_full: int, dim: int, batch: int, k: int, budget_s: float = 12.0) -> dict:
    """The reference's CPU path for this search: qdrant-client local mode COSINE (fp32 rows
    normalised at insert, fp32 dot, arg-selection), restated in numpy (oracle.dense_fp32_local)
    on a bounded sample of rows, batched B queries per GEMM; extrapolated linearly in rows."""
    from threadpoolctl import threadpool_limits

    from oracle import oracle

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    n_sample = 200_000
    rows = oracle.unit_fp16(n_sample, dim, seed=0)
    qs = oracle.unit_fp16(batch * 4, dim, seed=1)
    x = rows.view(np.float16).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    q = qs.view(np.float16).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    done = 0
    with threadpool_limits(limits=threads):
        s = q[:batch] @ x.T  # warm-up
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < budget_s:
            qb = q[(done % 4) * batch:(done % 4 + 1) * batch]
            s = qb @ x.T
            part = np.argpartition(-s, k, axis=1)[:, :k]
            np.take_along_axis(s, part, axis=1)
            done += 1
        el = time.perf_counter() - t0
    qps_sample = done * batch / el
    return {
        "value": qps_sample * n_sample / n_full,
        "unit": "queries/sec",
        "cores": threads,
        "kind": "port",
        "sample": (f"numpy fp32 normalised-dot + argpartition top-{k} (qdrant-client local-mode "
                   f"COSINE restated) over {n_sample} of the {n_full} rows, {done} batches of "
                   f"{batch} queries in {el:.1f}s on {threads} threads; qps scaled by "
                   f"{n_sample}/{n_full}"),
    }


def read_traffic() -> float | None:
    p = ROOT / "profiles" / "dense_scan_traffic.json"
    if p.exists():
        try:
            return float(json.loads(p.read_text())["hbm_bytes_per_launch"])
        except Exception:
            return None
    return None


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--chunks", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--top-k", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--latency-iters", type=int, default=30)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using {world}", file=sys.stderr)
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    distributed = world > 1
    if distributed:
        dist.init_process_group("nccl", device_id=dev)

    from audio_rag_amd import _armi
    from audio_rag_amd.retrieval.device import DenseIndex, merge_shards
    from audio_rag_amd.retrieval.shards import ShardedSearch, shard_range

    n, dim, batch, k = args.chunks, args.dim, args.batch, args.top_k
    lo, hi = shard_range(n, rank, world)
    rows = make_rows(lo, hi - lo, dim, dev)
    index = DenseIndex(rows, ordinal_base=lo)
    n_q_batches = 8
    queries = make_queries(n_q_batches, batch, dim, dev, seed=1 + rank)
    ws = torch.empty(index.workspace_bytes(world * batch, k), dtype=torch.uint8, device=dev)
    sharded = None
    if distributed:
        sharded = ShardedSearch(lambda q, kk: index.topk(q, kk, workspace=ws), merge_shards)

    def step(i: int, q_local: torch.Tensor | None = None):
        ql = q_local if q_local is not None else queries[i % n_q_batches]
        if sharded is None:
            return index.topk(ql, k, workspace=ws)
        return sharded.dense(ql, k)

    def barrier():
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()

    for i in range(args.warmup):
        step(i)
    barrier()
    _armi.call("armi_scan_timing_enable", 1)
    _armi.call("armi_scan_timing_read", _armi.ctypes.byref(_armi.ctypes.c_double()),
               _armi.ctypes.byref(_armi.ctypes.c_int64()))
    barrier()
    t0 = time.perf_counter()
    last = None
    for i in range(args.steps):
        last = step(i)
    barrier()
    elapsed = time.perf_counter() - t0
    tot_ms, launches = _armi.ctypes.c_double(), _armi.ctypes.c_int64()
    _armi.call("armi_scan_timing_read", _armi.ctypes.byref(tot_ms), _armi.ctypes.byref(launches))
    _armi.call("armi_scan_timing_enable", 0)
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    certified = None
    if last is not None and last.flags is not None:
        certified = float((last.flags == 1).float().mean().item())

    # p50 latency of one step (batch of 64 per GPU) and of a single query
    lat, lat1 = [], []
    for i in range(args.latency_iters):
        barrier()
        t1 = time.perf_counter()
        step(i)
        barrier()
        lat.append(time.perf_counter() - t1)
    for i in range(args.latency_iters):
        barrier()
        t1 = time.perf_counter()
        step(i, queries[i % n_q_batches][:1])
        barrier()
        lat1.append(time.perf_counter() - t1)

    if rank != 0:
        if distributed:
            dist.barrier()
            dist.destroy_process_group()
        return

    total_queries = world * batch * args.steps
    scan_avg_ms = tot_ms.value / max(launches.value, 1)
    shard_rows = hi - lo
    alg_bytes = shard_rows * dim * 2 + shard_rows * 4 + batch * dim * 2
    achieved = alg_bytes / (scan_avg_ms * 1e-3) / 1e9
    traffic = read_traffic()
    result = {
        "metric": METRIC,
        "value": total_queries / elapsed,
        "unit": "queries/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f16",
        "data": "synthetic: N(0,1) rows and queries L2-normalised then cast to fp16 (SURVEY.md §8(d)), resident in HBM",
        "config": {
            "workload": (f"dense cosine top-{k} over {n} x {dim} fp16 chunks sharded by ordinal over "
                         f"{world} GPU(s), {batch} queries per GPU per step (RCCL all-gather of "
                         f"queries and per-shard top-{k} when N>1)"),
            "n_chunks": n, "dim": dim, "batch_per_gpu": batch, "top_k": k,
            "parallelism": f"corpus-shard{world}",
        },
        "p50_ms": statistics.median(lat) * 1e3,
        "p50_single_query_ms": statistics.median(lat1) * 1e3,
        "certified_frac": certified,
        "roofline": {
            "bound": "hbm",
            "kernel": "dense_scan_kernel<1024>",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "algorithmic_bytes_per_launch": alg_bytes,
            "avg_launch_ms": scan_avg_ms,
            "launches_timed": launches.value,
        },
    }
    if world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(n, dim, batch, k)
    else:
        result["cpu_baseline"] = None
    print(json.dumps(result), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
