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

from audio_rag_amd.synthetic import (VOCAB, doc_tokens, make_queries, make_rows,  # noqa: E402
                                     make_sparse_queries, make_sparse_rows)

METRIC = json.loads((ROOT / "BASELINE.json").read_text())["metric"]
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
# dense (non-sparse) matrix peaks, MI355X_MICROARCH.md: bf16/f16 ~2.5 PF; fp32-input MFMA runs at
# 1/16 of the bf16 rate (cdna_hip_programming.md §3 'FP32-input MFMA')
MFMA_PEAK_TFLOPS = {"fp16": 2500.0, "bf16": 2500.0, "fp32": 157.0}


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
    ap.add_argument("--workload", choices=["dense", "hybrid", "hybrid_rerank", "stream", "pipeline"],
                    default="dense",
                    help="dense: BASELINE metric (default); hybrid: dense+sparse prefetch 2k + RRF "
                         "(configs[2] without rerank); hybrid_rerank: configs[2]: top-20 fused -> "
                         "cross-encoder -> top-k; stream: single queries arriving at --qps "
                         "(Poisson) through QueryBatcher -> MI355XRetriever, reference-shaped "
                         "results (configs[4]'s streaming query, 1 GPU); pipeline: "
                         "QueryPipeline.query() one query at a time (BGE-M3 encode -> hybrid "
                         "search -> rerank), per-stage latency beside the reference's published "
                         "numbers")
    ap.add_argument("--queries", type=int, default=200, help="pipeline: timed queries")
    ap.add_argument("--qps", type=float, default=20000.0, help="stream: offered queries/s")
    ap.add_argument("--duration", type=float, default=4.0, help="stream: seconds of arrivals")
    ap.add_argument("--initial-k", type=int, default=20)
    ap.add_argument("--rerank-dtype", choices=["fp32", "bf16", "fp16"], default="fp16",
                    help="cross-encoder GEMM dtype (fp16: fp16 GEMMs + fused fp16 attention, "
                         "within the 1e-3 score budget; fp32: the reference's dtype)")
    args = ap.parse_args()

    if args.workload == "stream":
        return stream_main(args)
    if args.workload == "pipeline":
        return pipeline_main(args)
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
    from audio_rag_amd.retrieval.device import (ConcurrentHybrid, DenseIndex, SparseIndex, TopK,
                                                merge_shards, rrf_fuse)
    from audio_rag_amd.retrieval.shards import ShardedSearch, shard_range

    n, dim, batch, k = args.chunks, args.dim, args.batch, args.top_k
    wl = args.workload
    search_k = k if wl == "dense" else (args.initial_k if wl == "hybrid_rerank" else k)
    pre_k = search_k if wl == "dense" else 2 * search_k
    lo, hi = shard_range(n, rank, world)
    rows = make_rows(lo, hi - lo, dim, dev)
    index = DenseIndex(rows, ordinal_base=lo)
    n_q_batches = 8
    queries = make_queries(n_q_batches, batch, dim, dev, seed=1 + rank)
    ws = torch.empty(index.workspace_bytes(world * batch, pre_k), dtype=torch.uint8, device=dev)
    sindex = None
    q_sparse = []
    if wl != "dense":
        sindex = SparseIndex(*make_sparse_rows(lo, hi - lo, dev), vocab=VOCAB, ordinal_base=lo)
        sws = torch.empty(sindex.workspace_bytes(world * batch, pre_k), dtype=torch.uint8, device=dev)
        q_sparse = [make_sparse_queries(batch, dev, seed=1000 * (1 + rank) + j) for j in range(n_q_batches)]
        hybrid = ConcurrentHybrid(dev)
    reranker = None
    if wl == "hybrid_rerank":
        from audio_rag_amd.reranking.xlmr import CrossEncoderXLMR, build_reranker
        reranker = CrossEncoderXLMR(build_reranker(seed=5), dev)
        if args.rerank_dtype != "fp32":
            reranker.to_dtype({"bf16": torch.bfloat16, "fp16": torch.float16}[args.rerank_dtype])
        gq = torch.Generator(device=dev).manual_seed(4 + rank)
        q_tokens = torch.randint(4, VOCAB, (n_q_batches, batch, 16), generator=gq, device=dev,
                                 dtype=torch.int32)
    sharded = None
    if distributed:
        sharded = ShardedSearch(lambda q, kk: index.topk(q, kk, workspace=ws), merge_shards,
                                local_sparse=(lambda c, kk: sindex.topk(*c, kk, workspace=sws)) if sindex else None,
                                rrf=lambda a, b, kk: rrf_fuse(a, b, kk))

    # live timing of the cross-encoder forward (runs on torch's current stream)
    rr_timing = {"on": False, "events": [], "flops": 0.0}

    def rerank(fused: TopK, qt: torch.Tensor) -> TopK:
        """configs[2]: every query's fused candidates -> (query, chunk) pairs of L = 256 tokens
        (<s> q16 </s></s> d236 </s>) -> cross-encoder -> stable sort -> top-k."""
        nb, kc = fused.ids.shape
        ids = fused.ids.clamp(min=0)
        d = doc_tokens(ids, 236)
        eos = torch.full((nb, kc, 1), 2, dtype=torch.int32, device=dev)
        bos = torch.zeros((nb, kc, 1), dtype=torch.int32, device=dev)
        qq = qt[:, None, :].expand(nb, kc, qt.shape[1])
        pairs = torch.cat([bos, qq, eos, eos, d, eos], dim=2).reshape(nb * kc, -1).contiguous()
        valid = (torch.arange(kc, device=dev)[None, :] < fused.count[:, None])
        mask = torch.ones_like(pairs)
        if rr_timing["on"]:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        probs = reranker.forward(pairs, mask).view(nb, kc)
        if rr_timing["on"]:
            ev[1].record()
            rr_timing["events"].append(ev)
            rr_timing["flops"] += reranker.flops(pairs.shape[0], pairs.shape[1])
        probs = torch.where(valid, probs, torch.full_like(probs, -1.0))
        order = torch.sort(probs, dim=1, descending=True, stable=True).indices[:, :k]
        return TopK(scores=torch.gather(probs, 1, order), ids=torch.gather(fused.ids, 1, order),
                    rank=torch.gather(probs, 1, order).double(),
                    count=torch.clamp(fused.count, max=k))

    def step(i: int, q_local: torch.Tensor | None = None):
        j = i % n_q_batches
        ql = q_local if q_local is not None else queries[j]
        if wl == "dense":
            if sharded is None:
                return index.topk(ql, k, workspace=ws)
            return sharded.dense(ql, k)
        qs = q_sparse[j]
        if ql.shape[0] != batch:  # single-query latency probe
            qs = (qs[0][:ql.shape[0] + 1], qs[1], qs[2])
        if sharded is None:
            fused = hybrid(lambda: index.topk(ql, pre_k, workspace=ws),
                           lambda: sindex.topk(*qs, pre_k, workspace=sws), qs, search_k)
        else:
            fused = sharded.hybrid(ql, qs, search_k)
        if reranker is None:
            return fused
        return rerank(fused, q_tokens[j][:ql.shape[0]])

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
    rr_timing["on"] = reranker is not None
    t0 = time.perf_counter()
    last = None
    for i in range(args.steps):
        last = step(i)
    barrier()
    elapsed = time.perf_counter() - t0
    rr_timing["on"] = False
    rr_ms = sum(a.elapsed_time(b) for a, b in rr_timing["events"])
    tot_ms, launches = _armi.ctypes.c_double(), _armi.ctypes.c_int64()
    _armi.call("armi_scan_timing_read", _armi.ctypes.byref(tot_ms), _armi.ctypes.byref(launches))
    _armi.call("armi_scan_timing_enable", 0)
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    certified = None
    if wl == "dense" and last is not None and last.flags is not None:
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
    nq_scan = world * batch  # queries each rank's scan processes per step (all-gathered)
    alg_bytes = shard_rows * dim * 2 + shard_rows * 4 + nq_scan * dim * 2
    alg_flops = 2.0 * shard_rows * dim * nq_scan
    # the scan's bound: HBM while the batch is small (arithmetic intensity ~ queries/pass flop/B),
    # the fp16 MFMA once the all-gathered batch of a multi-GPU step passes the ridge
    mfma_bound = alg_flops / (MFMA_PEAK_TFLOPS["fp16"] * 1e12) > alg_bytes / (HBM_PEAK_GBS * 1e9)
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
            "workload": {
                "dense": (f"dense cosine top-{k} over {n} x {dim} fp16 chunks sharded by ordinal over "
                          f"{world} GPU(s), {batch} queries per GPU per step (RCCL all-gather of "
                          f"queries and per-shard top-{k} when N>1)"),
                "hybrid": (f"hybrid top-{k}: dense cosine + sparse lexical prefetch {pre_k} each, RRF "
                           f"(1/(2+pos)), {n} chunks, {batch} queries per GPU per step"),
                "hybrid_rerank": (f"hybrid top-{search_k} (prefetch {pre_k}+{pre_k}, RRF) -> "
                                  f"cross-encoder (XLM-R base, 12 layers, L=256, "
                                  f"{args.rerank_dtype} GEMMs) -> top-{k}, {n} chunks, {batch} "
                                  f"queries per GPU per step"),
            }[wl],
            "n_chunks": n, "dim": dim, "batch_per_gpu": batch, "top_k": k,
            "parallelism": f"corpus-shard{world}",
        },
        "p50_ms": statistics.median(lat) * 1e3,
        "p50_single_query_ms": statistics.median(lat1) * 1e3,
        "certified_frac": certified,
        "roofline": ({
            "bound": "hbm",
            "kernel": ("dense_scan_kernel<1024>" if nq_scan <= 128
                       else "dense_gemm_scan_glds_kernel<1024>"),
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic if nq_scan <= 64 else None,
            "algorithmic_bytes_per_launch": alg_bytes,
            "avg_launch_ms": scan_avg_ms,
            "launches_timed": launches.value,
        } if not mfma_bound else {
            "bound": "mfma",
            "kernel": "dense_gemm_scan_glds_kernel<1024>",
            "achieved": alg_flops / (scan_avg_ms * 1e-3) / 1e12,
            "peak": MFMA_PEAK_TFLOPS["fp16"],
            "unit": "TFLOP/s",
            "frac": alg_flops / (scan_avg_ms * 1e-3) / 1e12 / MFMA_PEAK_TFLOPS["fp16"],
            "traffic": None,
            "algorithmic_flops_per_launch": alg_flops,
            "algorithmic_bytes_per_launch": alg_bytes,
            "hbm_gbs_achieved": achieved,
            "avg_launch_ms": scan_avg_ms,
            "launches_timed": launches.value,
        }),
    }
    if reranker is not None and rr_timing["events"]:
        # configs[2]: the cross-encoder is the dominant (MFMA-bound) stage; the scan roofline
        # moves to roofline_scan
        rr_tflops = rr_timing["flops"] / (rr_ms * 1e-3) / 1e12
        peak = MFMA_PEAK_TFLOPS[args.rerank_dtype]
        result["roofline_scan"] = result["roofline"]
        result["roofline"] = {
            "bound": "mfma",
            "kernel": f"cross-encoder forward ({args.rerank_dtype} GEMMs, fused attention)",
            "achieved": rr_tflops,
            "peak": peak,
            "unit": "TFLOP/s",
            "frac": rr_tflops / peak,
            "traffic": None,
            "algorithmic_flops_per_step": rr_timing["flops"] / max(len(rr_timing["events"]), 1),
            "avg_forward_ms": rr_ms / max(len(rr_timing["events"]), 1),
            "forwards_timed": len(rr_timing["events"]),
        }
        result["rerank_share_of_step"] = (rr_ms * 1e-3) / elapsed
    if world == 1 and not args.no_cpu_baseline and wl == "dense":
        result["cpu_baseline"] = cpu_baseline(n, dim, batch, k)
    else:
        result["cpu_baseline"] = None
    print(json.dumps(result), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


WORDS = ("gradient descent learning rate loss function model training data neural network layer "
         "weights bias optimizer batch epoch regression classification feature vector matrix "
         "probability distribution bayes kernel margin support vector tree boosting variance "
         "lecture professor example equation derivative convex objective parameter sample").split()


def pipeline_main(args) -> None:
    """The reference's query path one query at a time, as AudioRAG.query() runs it
    (pipeline/query.py:97-215): BGE-M3 query encode (XLM-R large, 24 layers, fp16, HIP-graph
    replay), hybrid search (dense + sparse prefetch 2 x initial_k = 40 each, RRF -> 20) over the
    chunk store, cross-encoder rerank 20 -> 5 (XLM-R base, fp16), RetrievalResult objects; answer
    generation off. Weights are seeded (no checkpoints offline), so only timing is meaningful.
    value = 1 / mean end-to-end latency (one stream); the reference publishes single-GPU
    latencies for the same stages (on a ~100s-of-chunks corpus)."""
    import logging

    from audio_rag_amd.config.schema import AudioRAGConfig
    from audio_rag_amd.embeddings.bge_m3 import BGEM3Embedder
    from audio_rag_amd.pipeline.query import QueryPipeline
    from audio_rag_amd.reranking.bge import BGEReranker
    from audio_rag_amd.retrieval.collection import ChunkCollection
    from audio_rag_amd.retrieval.device import DenseIndex, SparseIndex
    from audio_rag_amd.retrieval.mi355x import MI355XRetriever

    logging.disable(logging.INFO)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n, dim = args.chunks, args.dim
    cfg = AudioRAGConfig()
    cfg.retrieval.search_type = "hybrid"
    rng = np.random.default_rng(11)
    texts = [" ".join(rng.choice(WORDS, size=int(rng.integers(30, 60)))) for _ in range(4096)]
    payloads = [{"text": texts[i % 4096], "start": float(i), "end": float(i) + 30.0,
                 "speaker": None, "metadata": {}} for i in range(n)]
    rows = make_rows(0, n, dim, dev)
    sindex = SparseIndex(*make_sparse_rows(0, n, dev), vocab=VOCAB)
    ret = MI355XRetriever(cfg.retrieval, dim)
    ret.attach_collection(ChunkCollection.from_indexes(cfg.retrieval.collection_name,
                                                       DenseIndex(rows), payloads, sindex))
    emb = BGEM3Embedder(cfg.embedding, device=dev)
    emb.load()
    rr = BGEReranker(cfg.reranking, device=dev)
    rr.load()
    pipe = QueryPipeline(cfg)
    pipe._embedder, pipe._retriever = emb, ret
    pipe._reranker, pipe._reranker_created = rr, True
    queries = [" ".join(rng.choice(WORDS, size=int(rng.integers(6, 16)))) for _ in range(256)]

    def sync_time(fn):
        torch.cuda.synchronize()
        t = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        return out, time.perf_counter() - t

    for q in queries[:16]:  # warm-up: graph capture per length bucket, kernel autotuning
        pipe.query(q, generate_answer=False)
    e2e, t_emb, t_search, t_rerank = [], [], [], []
    for i in range(args.queries):
        q = queries[i % len(queries)]
        res, t = sync_time(lambda: pipe.query(q, generate_answer=False))
        assert res.reranked and len(res.results) == cfg.reranking.top_k
        e2e.append(t)
        e, t = sync_time(lambda: emb.embed_query(q))
        t_emb.append(t)
        hits, t = sync_time(lambda: ret.search(e, top_k=cfg.reranking.initial_k,
                                               search_type="hybrid"))
        t_search.append(t)
        _, t = sync_time(lambda: rr.rerank(q, hits, top_k=cfg.reranking.top_k))
        t_rerank.append(t)
    ms = lambda xs, p: float(np.percentile(np.array(xs) * 1e3, p))
    print(json.dumps({
        "metric": METRIC,
        "value": 1.0 / float(np.mean(e2e)),
        "unit": "queries/sec",
        "n_gpus": 1,
        "steps": args.queries,
        "warmup": 16,
        "ms_per_step": float(np.mean(e2e)) * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f16",
        "data": ("synthetic: seeded BGE-M3 / reranker weights, N(0,1) unit fp16 chunk vectors, "
                 "Zipf sparse vectors, synthetic chunk and query texts"),
        "config": {"workload": (f"QueryPipeline.query() single-stream: BGE-M3 encode -> hybrid "
                                f"search (prefetch 40 + 40, RRF 20) over {n} chunks -> rerank "
                                f"20 -> 5 (fp16), one query at a time"),
                   "n_chunks": n, "dim": dim, "initial_k": cfg.reranking.initial_k,
                   "top_k": cfg.reranking.top_k, "parallelism": "single GPU, batch 1"},
        "p50_ms": ms(e2e, 50), "p95_ms": ms(e2e, 95), "p99_ms": ms(e2e, 99),
        "stage_p50_ms": {"embed": ms(t_emb, 50), "hybrid_search": ms(t_search, 50),
                         "rerank": ms(t_rerank, 50)},
        "reference_published_p50_ms": {"embed": 18, "hybrid_search": 48, "rerank": 38,
                                       "warm_query": 141,
                                       "source": "docs/SALES_TECHNICAL_GUIDE.md:563-565, "
                                                 "README.md:37-38 (single unspecified GPU, "
                                                 "~100s of chunks)"},
        "roofline": None,
        "cpu_baseline": None,
    }), flush=True)


def stream_main(args) -> None:
    """configs[4]'s query side on one GPU: single queries arrive as a Poisson process at
    --qps from a client thread, QueryBatcher coalesces them (<= 64 per batch, <= 2 ms wait) into
    MI355XRetriever.search_batch over the 1M-chunk store, and each caller gets its
    list[RetrievalResult]. value = completed queries / s; latency = submit -> result."""
    from audio_rag_amd.config import RetrievalConfig
    from audio_rag_amd.retrieval.batcher import QueryBatcher
    from audio_rag_amd.retrieval.collection import ChunkCollection
    from audio_rag_amd.retrieval.device import DenseIndex
    from audio_rag_amd.retrieval.mi355x import MI355XRetriever

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    # the client thread and the batcher thread share one interpreter: hand the GIL over at
    # 0.2 ms instead of the 5 ms default, or a batch waits for the client's time slice
    sys.setswitchinterval(2e-4)
    n, dim, k = args.chunks, args.dim, args.top_k
    rows = make_rows(0, n, dim, dev)
    payloads = [{"text": "", "start": 0.0, "end": 0.0, "speaker": None, "metadata": {}}] * n
    ret = MI355XRetriever(RetrievalConfig(top_k=k, search_type="dense"), dim)
    ret.attach_collection(ChunkCollection.from_indexes("audio_rag", DenseIndex(rows), payloads))
    qs = make_queries(1, 4096, dim, dev, seed=1)[0].cpu().numpy()
    rng = np.random.default_rng(7)
    lat, done = [], []
    lock = __import__("threading").Lock()

    def on_done(t_sub):
        def cb(f):
            t = time.perf_counter()
            f.result()
            with lock:
                lat.append(t - t_sub)
                done.append(t)
        return cb

    with QueryBatcher(ret, max_batch=64, max_wait_ms=2.0) as qb:
        for i in range(256):  # warm-up
            qb.submit_arrays(qs[i % 4096]).result()
        lat.clear()
        done.clear()
        n_q = int(args.qps * args.duration)
        gaps = rng.exponential(1.0 / args.qps, size=n_q)
        t0 = time.perf_counter()
        t_next = t0
        futs = []
        for i in range(n_q):
            t_next += gaps[i]
            delay = t_next - time.perf_counter()
            if delay > 0:
                time.sleep(delay)  # releases the GIL to the batcher thread (never spin here)
            f = qb.submit_arrays(qs[i % 4096])
            f.add_done_callback(on_done(time.perf_counter()))
            futs.append(f)
        for f in futs:
            f.result()
        batches, served = qb.batches, qb.queries
    t_end = max(done)
    value = len(done) / (t_end - t0)
    lat_ms = np.array(lat) * 1e3
    print(json.dumps({
        "metric": METRIC,
        "value": value,
        "unit": "queries/sec",
        "n_gpus": 1,
        "steps": batches,
        "warmup": 256,
        "ms_per_step": (t_end - t0) / max(batches, 1) * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f16",
        "data": "synthetic: N(0,1) rows and queries L2-normalised then cast to fp16, resident in HBM",
        "config": {"workload": (f"streaming dense top-{k}: Poisson arrivals at {args.qps:.0f} q/s "
                                f"for {args.duration:.1f} s, QueryBatcher (<=64, <=2 ms) -> "
                                f"MI355XRetriever.search_batch over {n} x {dim} fp16 chunks -> "
                                f"list[RetrievalResult] per caller"),
                   "n_chunks": n, "dim": dim, "top_k": k, "offered_qps": args.qps,
                   "parallelism": "single GPU, one batcher thread"},
        "p50_ms": float(np.percentile(lat_ms, 50)),
        "p99_ms": float(np.percentile(lat_ms, 99)),
        "mean_batch": served / max(batches, 1),
        "roofline": None,
        "cpu_baseline": None,
    }), flush=True)


if __name__ == "__main__":
    main()
