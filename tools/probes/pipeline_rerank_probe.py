"""Probe: the cross-encoder's first graphed call inside the AudioRAG pipeline against the eager
forward, with the retriever's / BGE-M3's query graphs and the shared capture pool switched by
argv flags (debugging the query() vs query_batch() rerank agreement)."""
import sys
import tempfile
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from ckpt_util import WORDS, save_bge_m3, save_reranker  # noqa: E402

from audio_rag_amd import AudioRAG  # noqa: E402
from audio_rag_amd.config import AudioRAGConfig  # noqa: E402
from audio_rag_amd.core import AudioChunk  # noqa: E402

pool, rgraph, egraph, batch_first = (int(x) for x in sys.argv[1:5])
if not pool:
    torch.cuda.graph_pool_handle = lambda: None
V = len(WORDS) + 4
d = Path(tempfile.mkdtemp())
save_bge_m3(d / "m3", 7, dict(vocab_size=V, num_hidden_layers=2))
save_reranker(d / "rr", 9, dict(vocab_size=V, num_hidden_layers=2))


def texts(n, seed, lo, hi):
    rng = np.random.default_rng(seed)
    return [" ".join(rng.choice(WORDS, size=int(rng.integers(lo, hi)))) for _ in range(n)]


cfg = AudioRAGConfig(embedding=dict(model=str(d / "m3"), query_graphs=bool(egraph)),
                     retrieval=dict(query_graphs=bool(rgraph)),
                     reranking=dict(model=str(d / "rr")),
                     generation=dict(backend="none"), log_level="WARNING")
rag = AudioRAG(cfg)
chunks = [AudioChunk(text=t, start=float(i), end=i + 1.0, speaker=None, metadata={"lecture": i % 3})
          for i, t in enumerate(texts(400, 5, 4, 30))]
rag.add_chunks(chunks)
queries = texts(12, 6, 2, 8)
rr = rag.query_pipeline.reranker
if batch_first:
    rag.query_batch(queries, search_type="hybrid", enable_reranking=True)
q = queries[0]
cands = rag.query(q, search_type="hybrid", enable_reranking=False, generate_answer=False, top_k=20).results
ct = [r.chunk.text for r in cands]
mode = sys.argv[5] if len(sys.argv) > 5 else ""
if mode == "eager_first":
    rr.load()
    rr._model.use_graphs = False
if mode == "load_first":
    rr.load()
    torch.cuda.synchronize()
orig_replay = torch.cuda.CUDAGraph.replay
if mode in ("sync", "twice"):
    def replay(self, _o=orig_replay, _m=mode):
        if _m == "sync":
            torch.cuda.synchronize()
        _o(self)
        if _m == "twice":
            _o(self)
    torch.cuda.CUDAGraph.replay = replay
a = np.array(rr.score_pairs(q, ct))
torch.cuda.CUDAGraph.replay = orig_replay
rr._model.use_graphs = True
b = np.array(rr.score_pairs(q, ct))
rr._model.use_graphs = False
e = np.array(rr.score_pairs(q, ct))
print(f"pool {pool} rgraph {rgraph} egraph {egraph} batch_first {batch_first}: "
      f"first-vs-eager {np.abs(a - e).max():.2e} second-vs-eager {np.abs(b - e).max():.2e}")

# second experiment: a fresh reranker object in the same process; first call with a sync
# between the input writes and the replay, then replayed twice
from audio_rag_amd.reranking.bge import BGEReranker  # noqa: E402
from audio_rag_amd.text import pair_ids  # noqa: E402

for mode in ("plain", "sync", "twice"):
    r2 = BGEReranker(cfg.reranking, device=torch.device("cuda", 0))
    r2.load()
    m = r2._model
    orig_replay = torch.cuda.CUDAGraph.replay

    def replay(self, _o=orig_replay, _m=mode):
        if _m == "sync":
            torch.cuda.synchronize()
        _o(self)
        if _m == "twice":
            _o(self)

    torch.cuda.CUDAGraph.replay = replay
    qt = r2.tokenizer.tokenize(q)
    pairs = [pair_ids(qt, r2.tokenizer.tokenize(t), 512) for t in ct]
    a2 = r2.score_ids(pairs).cpu().numpy()
    torch.cuda.CUDAGraph.replay = orig_replay
    m.use_graphs = False
    e2 = r2.score_ids(pairs).cpu().numpy()
    print(f"fresh reranker, {mode}: first-vs-eager {np.abs(a2 - e2).max():.2e}")
