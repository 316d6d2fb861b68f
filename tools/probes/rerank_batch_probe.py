"""Probe: cross-encoder scores of the same pairs scored alone (20 pairs) and inside a larger
batch, graphed and eager (debugging the query() vs query_batch() rerank agreement)."""
import sys
import tempfile
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "tests"))
from ckpt_util import WORDS, save_reranker  # noqa: E402

from audio_rag_amd.config.schema import RerankingConfig  # noqa: E402
from audio_rag_amd.reranking.bge import BGEReranker  # noqa: E402
from audio_rag_amd.text import pair_ids  # noqa: E402

V = len(WORDS) + 4
d = Path(tempfile.mkdtemp())
save_reranker(d / "rr", 9, dict(vocab_size=V, num_hidden_layers=2))
rr = BGEReranker(RerankingConfig(model=str(d / "rr")), device=torch.device("cuda", 0))
rr.load()
rng = np.random.default_rng(5)
texts = [" ".join(rng.choice(WORDS, size=int(rng.integers(4, 30)))) for _ in range(240)]
q = rr.tokenizer.tokenize("search search rate cache")
pairs = [pair_ids(q, rr.tokenizer.tokenize(t), 512) for t in texts]
for graphs in (True, False):
    rr._model.use_graphs = graphs
    a = rr.score_ids(pairs[:20]).cpu().numpy()
    b = rr.score_ids(pairs).cpu().numpy()[:20]
    print("graphs", graphs, "max |alone - batch|", float(np.abs(a - b).max()))
    print(" alone", np.round(a[:8], 4))
    print(" batch", np.round(b[:8], 4))
