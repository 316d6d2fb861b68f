"""Single-query latency of MI355XRetriever.search (the reference-shaped call AudioRAG.query()
issues, pipeline/query.py:152-167) split into its host/device stages, at 1M chunks:
to_query_batch (host -> device query), search_batch (the kernels, synchronised), materialize
(device -> host + RetrievalResult objects), and the whole search(). p50 over --iters calls."""
import argparse
import json
import statistics
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from audio_rag_amd.config import RetrievalConfig  # noqa: E402
from audio_rag_amd.core import EmbeddingResult, SparseVector  # noqa: E402
from audio_rag_amd.retrieval.collection import ChunkCollection  # noqa: E402
from audio_rag_amd.retrieval.device import DenseIndex, SparseIndex  # noqa: E402
from audio_rag_amd.retrieval.mi355x import MI355XRetriever  # noqa: E402
from audio_rag_amd.synthetic import (VOCAB, make_queries, make_rows, make_sparse_queries,  # noqa: E402
                                     make_sparse_rows)


def p50(xs):
    return statistics.median(xs) * 1e3


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--top-k", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = args.chunks
    rows = make_rows(0, n, 1024, dev)
    sidx = SparseIndex(*make_sparse_rows(0, n, dev), vocab=VOCAB)
    payloads = [{"text": "", "start": 0.0, "end": 30.0, "speaker": None, "metadata": {}}] * n
    ret = MI355XRetriever(RetrievalConfig(search_type="hybrid"), 1024)
    ret.attach_collection(ChunkCollection.from_indexes("audio_rag", DenseIndex(rows), payloads,
                                                       sidx))
    qd = make_queries(1, 256, 1024, dev, seed=1)[0].float().cpu().numpy()
    qp, qi, qv = (t.cpu().numpy() for t in make_sparse_queries(256, dev, seed=1000))
    embs = [EmbeddingResult(dense=qd[i].tolist(),
                            sparse=SparseVector(qi[qp[i]:qp[i + 1]].tolist(),
                                                qv[qp[i]:qp[i + 1]].tolist())) for i in range(256)]
    out = {}
    for st in ("hybrid", "dense"):
        t_q, t_s, t_m, t_all = [], [], [], []
        for it in range(args.iters + 20):
            e = embs[it % 256]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = ret.search(e, top_k=args.top_k, search_type=st)
            t1 = time.perf_counter()
            b = ret.to_query_batch([e])
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            o, mode = ret.search_batch(b, args.top_k, "audio_rag", None, st)
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            ret.materialize(o, mode, "audio_rag", 0, None)
            t4 = time.perf_counter()
            assert len(res) == args.top_k
            if it >= 20:
                t_all.append(t1 - t0)
                t_q.append(t2 - t1)
                t_s.append(t3 - t2)
                t_m.append(t4 - t3)
        out[st] = {"search_p50_ms": p50(t_all), "to_query_batch_p50_ms": p50(t_q),
                   "search_batch_p50_ms": p50(t_s), "materialize_p50_ms": p50(t_m)}
    print(json.dumps({"chunks": n, "top_k": args.top_k, "iters": args.iters, **out}, indent=1))


if __name__ == "__main__":
    main()
