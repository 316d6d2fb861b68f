"""Probe: the cross-encoder's first graphed call (capture + replay) against the second and the
eager forward, with and without the shared capture pool and the pair-count bucket."""
import sys
import tempfile
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from ckpt_util import WORDS, save_reranker  # noqa: E402

from audio_rag_amd.config.schema import RerankingConfig  # noqa: E402
from audio_rag_amd.reranking.bge import BGEReranker  # noqa: E402
from audio_rag_amd.reranking.xlmr import CrossEncoderXLMR  # noqa: E402
from audio_rag_amd.text import pair_ids  # noqa: E402

V = len(WORDS) + 4
d = Path(tempfile.mkdtemp())
save_reranker(d / "rr", 9, dict(vocab_size=V, num_hidden_layers=2))
rng = np.random.default_rng(5)
texts = [" ".join(rng.choice(WORDS, size=int(rng.integers(4, 30)))) for _ in range(20)]
for pool, bucket in ((True, True), (False, True), (True, False), (False, False)):
    rr = BGEReranker(RerankingConfig(model=str(d / "rr")), device=torch.device("cuda", 0))
    rr.load()
    m = rr._model
    if not bucket:
        m._n_bucket = staticmethod(lambda n: n)
    if not pool:
        m._pool = None
        orig = torch.cuda.graph_pool_handle
        torch.cuda.graph_pool_handle = lambda: None
    q = rr.tokenizer.tokenize("search search rate cache")
    pairs = [pair_ids(q, rr.tokenizer.tokenize(t), 512) for t in texts]
    a = rr.score_ids(pairs).cpu().numpy()
    b = rr.score_ids(pairs).cpu().numpy()
    m.use_graphs = False
    e = rr.score_ids(pairs).cpu().numpy()
    if not pool:
        torch.cuda.graph_pool_handle = orig
    print(f"pool {pool} bucket {bucket}: first-vs-eager {np.abs(a - e).max():.2e} "
          f"second-vs-eager {np.abs(b - e).max():.2e}")
