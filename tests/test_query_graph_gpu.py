"""search() of one unfiltered query through the collection's captured HIP graph (_QueryGraph):
its answers must equal search_batch's for every branch (dense / sparse-only / hybrid, several
top_k, the staging buffer reused across queries), and the graph must capture in a process whose
reranker captured its own forward graph first (and the reverse order), as AudioRAG.query() does
them (pipeline/query.py:131-198): both captures share the CUDA generator's graph state.
Each ordering runs in its own spawned process, since that state lives for the process.
Reference: QdrantRetriever.search (retrieval/qdrant.py:227-352)."""

import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent
N, DIM, B = 5000, 1024, 6


def _worker(order, out_dir):
    sys.path.insert(0, str(ROOT))
    torch.cuda.set_device(0)
    from audio_rag_amd.config import RetrievalConfig
    from audio_rag_amd.config.schema import RerankingConfig
    from audio_rag_amd.core import EmbeddingResult, SparseVector
    from audio_rag_amd.reranking.bge import BGEReranker
    from audio_rag_amd.retrieval.mi355x import MI355XRetriever
    from oracle import oracle as o

    rows = o.unit_fp16(N, DIM, seed=41)
    ip, ix, iv = o.sparse_corpus(N, seed=42)
    sparse = [(ix[ip[r]:ip[r + 1]], iv[ip[r]:ip[r + 1]]) for r in range(N)]
    payloads = [{"text": f"chunk {r} words{r % 13}", "start": float(r), "end": r + 1.0,
                 "speaker": None, "metadata": {}} for r in range(N)]
    ret = MI355XRetriever(RetrievalConfig(top_k=5), DIM)
    ret.add_arrays(rows.view(np.float16), payloads, sparse=sparse)
    coll = ret.collection()
    qd = o.unit_fp16(B, DIM, seed=43).view(np.float16).astype(np.float32)
    qi, qx, qv = o.sparse_queries(B, seed=44)
    embs = [EmbeddingResult(dense=qd[i].tolist(),
                            sparse=SparseVector(qx[qi[i]:qi[i + 1]].tolist(),
                                                qv[qi[i]:qi[i + 1]].tolist())) for i in range(B)]
    rr = BGEReranker(RerankingConfig(top_k=3), device=torch.device("cuda", 0),
                     arch=dict(num_hidden_layers=1))
    rr.load()

    def rerank():
        hits = ret.search_batch(ret.to_query_batch(embs[:1]), 5, None, None, "dense")
        res = ret.materialize_batch(*hits, coll.name)[0]
        return [r.score for r in rr.rerank("query", res)]

    if order == "rerank_first":
        rerank()
    bad = []
    for st in ("dense", "sparse", "hybrid"):
        for k in (1, 5, 20):
            for e in embs:
                got = ret.search(e, top_k=k, search_type=st)
                tk, mode = ret.search_batch(ret.to_query_batch([e]), k, None, None, st)
                want = ret.materialize_batch(tk, mode, coll.name)[0]
                if ([(r.chunk.text, r.score) for r in got]
                        != [(r.chunk.text, r.score) for r in want]):
                    bad.append((st, k))
    if order == "search_first":
        rerank()
    np.savez(Path(out_dir) / f"{order}.npz", bad=np.array(len(bad)),
             graphs=np.array(len(coll.query_graphs())), ok=np.array(ret._graphs_ok))


@pytest.mark.parametrize("order", ["rerank_first", "search_first"])
def test_query_graph_equals_batch_path(tmp_path, order):
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_worker, args=(order, str(tmp_path)))
    p.start()
    p.join(240)
    if p.is_alive():
        p.kill()
        p.join()
    assert p.exitcode == 0, p.exitcode
    z = np.load(tmp_path / f"{order}.npz")
    assert bool(z["ok"]), "the query graph capture was refused"
    assert int(z["graphs"]) == 9  # one per (branch, top_k)
    assert int(z["bad"]) == 0
