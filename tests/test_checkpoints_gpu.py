"""Checkpoints on disk drive the encoders (audio_rag_amd/checkpoints.py) and the query encode is
one arithmetic for query() and query_batch().

Seeded BGE-M3 / bge-reranker-base twins (2 layers, a 36-word vocabulary) are saved with
save_pretrained (model.safetensors), BGE-M3's sparse_linear.pt and a tokenizer.json; load() on
config.model = that directory must reproduce the seeded path's vectors, lexical weights and
scores bit for bit, and tokenise with the tokenizer.json. Then AudioRAG over those checkpoints:
query() and query_batch() return identical results for the same texts.
Reference: BGEM3FlagModel(config.model) (embeddings/bge.py:47-55), CrossEncoder(config.model)
(reranking/bge.py:50-55), AudioRAG.query (pipeline/query.py:97-215)."""

import sys
from pathlib import Path

import numpy as np
import pytest
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
from ckpt_util import WORDS, save_bge_m3, save_reranker  # noqa: E402

pytestmark = pytest.mark.gpu
V = len(WORDS) + 4
M3 = dict(vocab_size=V, num_hidden_layers=2)
RR = dict(vocab_size=V, num_hidden_layers=2)


@pytest.fixture(scope="module")
def ckpts(tmp_path_factory):
    root = tmp_path_factory.mktemp("ckpt")
    save_bge_m3(root / "m3", 7, M3)
    save_reranker(root / "rr", 9, RR)
    return root


def _texts(n, seed, lo=3, hi=12):
    rng = np.random.default_rng(seed)
    return [" ".join(rng.choice(WORDS, size=int(rng.integers(lo, hi)))) for _ in range(n)]


def test_loaded_encoders_equal_seeded_twins(gpu, ckpts):
    from audio_rag_amd.checkpoints import HFTokenizer
    from audio_rag_amd.config.schema import EmbeddingConfig, RerankingConfig
    from audio_rag_amd.embeddings.bge_m3 import BGEM3Embedder
    from audio_rag_amd.reranking.bge import BGEReranker

    loaded = BGEM3Embedder(EmbeddingConfig(model=str(ckpts / "m3")), device=gpu)
    loaded.load()
    seeded = BGEM3Embedder(EmbeddingConfig(model="absent/bge-m3", seed=7), device=gpu, arch=M3)
    seeded.load()
    assert isinstance(loaded.tokenizer, HFTokenizer) and loaded.dimension == 1024
    for text in _texts(6, 1) + ["lecture " * 40]:
        ids = loaded.tokenizer.encode(text)
        assert ids[0] == 0 and ids[-1] == 2 and all(3 <= i < V for i in ids[1:-1])
        a, la = loaded.encode_query_ids(ids)
        b, lb = seeded.encode_query_ids(ids)
        assert torch.equal(a, b) and la == lb
        assert loaded.embed_query(text).dense == a[0].float().cpu().tolist()
    ea = loaded.embed(_texts(5, 2))
    ids = [loaded.tokenizer.encode(t) for t in _texts(5, 2)]
    da, _ = loaded.encode_ids(ids)
    db, _ = seeded.encode_ids(ids)
    assert torch.equal(da, db) and len(ea) == 5
    rl = BGEReranker(RerankingConfig(model=str(ckpts / "rr")), device=gpu)
    rs = BGEReranker(RerankingConfig(model="absent/reranker", seed=9), device=gpu, arch=RR)
    rl.load()
    rs.load()
    q = rl.tokenizer.tokenize("gradient descent learning rate")
    from audio_rag_amd.text import pair_ids

    pairs = [pair_ids(q, rl.tokenizer.tokenize(t), 512) for t in _texts(20, 3)]
    assert torch.equal(rl.score_ids(pairs), rs.score_ids(pairs))
    assert rl.score_pairs("gradient descent learning rate", _texts(20, 3)) == \
        rs.score_ids(pairs).cpu().tolist()


def test_batched_query_encode_equals_single(gpu, ckpts):
    """embed_queries (QueryPipeline.query_batch's encode) gives every query exactly the dense
    vector and lexical weights embed_query (the captured batch-1 graph) gives it: the armi query
    encoder's arithmetic is row-independent (linears in 32-row blocks, per-row normalisation)."""
    from audio_rag_amd.config.schema import EmbeddingConfig
    from audio_rag_amd.embeddings.bge_m3 import BGEM3Embedder

    e = BGEM3Embedder(EmbeddingConfig(model=str(ckpts / "m3")), device=gpu)
    e.load()
    texts = _texts(37, 4, 1, 40) + ["lecture " * 70]  # 1 .. 72 tokens: buckets 16 .. 128
    dense, lex = e.embed_queries(texts)
    for i, t in enumerate(texts):
        one = e.embed_query(t)
        assert one.dense == dense[i].float().cpu().tolist(), i
        want = e._convert_sparse(lex[i])
        assert (one.sparse is None and want is None) or (one.sparse.indices == want.indices
                                                         and one.sparse.values == want.values), i


def test_pipeline_query_and_query_batch_agree(gpu, ckpts):
    from audio_rag_amd import AudioRAG
    from audio_rag_amd.config import AudioRAGConfig
    from audio_rag_amd.core import AudioChunk

    cfg = AudioRAGConfig(embedding=dict(model=str(ckpts / "m3")),
                         reranking=dict(model=str(ckpts / "rr")),
                         generation=dict(backend="none"), log_level="WARNING")
    rag = AudioRAG(cfg)
    chunks = [AudioChunk(text=t, start=float(i), end=i + 1.0, speaker=None,
                         metadata={"lecture": i % 3}) for i, t in enumerate(_texts(400, 5, 4, 30))]
    rag.add_chunks(chunks)
    queries = _texts(12, 6, 2, 8)
    for st in ("hybrid", "dense", "sparse"):
        for rerank in (False, True):
            batch = rag.query_batch(queries, search_type=st, enable_reranking=rerank)
            for q, b in zip(queries, batch):
                one = rag.query(q, search_type=st, enable_reranking=rerank, generate_answer=False)
                got = [(r.chunk.start, r.score) for r in one.results]
                want = [(r.chunk.start, r.score) for r in b.results]
                if not rerank:
                    assert got == want, (st, q)
                else:
                    # the cross-encoder scores pairs in batches of different sizes (20 vs 240):
                    # its GEMMs agree to ~1e-5, so the sorted scores agree position by position
                    # and the ids wherever the neighbouring scores are further apart than that
                    # (a 2-layer random model scores every pair 0.48 +- 0.01: near-ties abound)
                    gs, ws = [g[1] for g in got], [w[1] for w in want]
                    assert len(gs) == len(ws)
                    np.testing.assert_allclose(gs, ws, rtol=0, atol=1e-4)
                    for i in range(len(gs)):
                        gap = min([abs(gs[i] - gs[j]) for j in (i - 1, i + 1) if 0 <= j < len(gs)]
                                  + [1.0])
                        if gap > 2e-4:
                            assert got[i][0] == want[i][0], (st, q, i)
