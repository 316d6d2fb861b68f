"""Cross-encoder (bge-reranker-base shape) and BGE-M3 encoder on the GPU.

Per-kernel numerics: each armi_enc_* kernel against a plain PyTorch fp32 reference of the same op
(tolerance 1e-5 absolute on O(1) activations). End to end: CrossEncoderXLMR against transformers'
XLMRobertaForSequenceClassification (fp32, CPU, same seeded weights) + sigmoid, tolerance 1e-3 on
the score (north_star: "rerank scores within 1e-3")."""

import math
from pathlib import Path

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _call(name, *args):
    from audio_rag_amd._armi import call, stream_handle

    call(name, *args, stream_handle())
    torch.cuda.synchronize()


def test_layernorm_residual(gpu):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(300, 768, generator=g)
    r = torch.randn(300, 768, generator=g)
    w = torch.randn(768, generator=g)
    b = torch.randn(768, generator=g)
    ref = torch.nn.functional.layer_norm(x + r, (768,), w, b, 1e-5)
    X, R, W, B = (t.to(gpu) for t in (x, r, w, b))
    out = torch.empty_like(X)
    _call("armi_enc_layernorm_residual", X.data_ptr(), R.data_ptr(), W.data_ptr(), B.data_ptr(),
          out.data_ptr(), 300, 768, 1e-5)
    torch.testing.assert_close(out.cpu(), ref, rtol=0, atol=2e-5)
    _call("armi_enc_layernorm_residual", X.data_ptr(), None, W.data_ptr(), B.data_ptr(),
          out.data_ptr(), 300, 768, 1e-5)
    torch.testing.assert_close(out.cpu(), torch.nn.functional.layer_norm(x, (768,), w, b, 1e-5),
                               rtol=0, atol=2e-5)


@pytest.mark.parametrize("L", [7, 64, 256, 512])
def test_masked_softmax(gpu, L):
    g = torch.Generator().manual_seed(L)
    n, H = 3, 4
    s = torch.randn(n, H, L, L, generator=g) * 4
    lens = [L, max(1, L // 2), 1]
    mask = torch.zeros(n, L, dtype=torch.int32)
    for i, ln in enumerate(lens):
        mask[i, :ln] = 1
    scale = 1 / math.sqrt(64)
    add = (1 - mask.float())[:, None, None, :] * torch.finfo(torch.float32).min
    ref = torch.softmax(s * scale + add, dim=-1)
    S = s.to(gpu).contiguous()
    M = mask.to(gpu)
    _call("armi_enc_masked_softmax", S.data_ptr(), M.data_ptr(), n, H, L, scale)
    torch.testing.assert_close(S.cpu(), ref, rtol=0, atol=1e-6)


def test_bias_gelu(gpu):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(128, 3072, generator=g) * 3
    b = torch.randn(3072, generator=g)
    ref = torch.nn.functional.gelu(x + b)
    X = x.to(gpu).contiguous()
    Bd = b.to(gpu)
    _call("armi_enc_bias_gelu", X.data_ptr(), Bd.data_ptr(), 128, 3072)
    torch.testing.assert_close(X.cpu(), ref, rtol=0, atol=1e-5)


def test_embed_positions_and_layernorm(gpu):
    g = torch.Generator().manual_seed(2)
    V, P, d = 1000, 80, 768
    word = torch.randn(V, d, generator=g)
    pos = torch.randn(P, d, generator=g)
    typ = torch.randn(d, generator=g)
    w, b = torch.randn(d, generator=g), torch.randn(d, generator=g)
    ids = torch.randint(4, V, (3, 40), generator=g)
    ids[0, 30:] = 1
    ids[2, 5:] = 1
    ids[1, 10] = 1  # an interior pad
    nonpad = ids.ne(1).int()  # XLM-R: padding_idx + running count of non-pad tokens
    pid = torch.cumsum(nonpad, dim=1) * nonpad + 1
    ref = torch.nn.functional.layer_norm(word[ids] + pos[pid] + typ, (d,), w, b, 1e-5)
    out = torch.empty(3 * 40, d, device=gpu)
    dev = [t.to(gpu).contiguous() for t in (ids.int(), word, pos, typ, w, b)]  # keep alive
    _call("armi_enc_embed", *(t.data_ptr() for t in dev), out.data_ptr(), 3, 40, d, 1, V, P, 1e-5)
    torch.testing.assert_close(out.cpu().view(3, 40, d), ref, rtol=0, atol=2e-5)


def _hf_scores(model, ids, mask):
    with torch.no_grad():
        return torch.sigmoid(model(input_ids=ids, attention_mask=mask).logits[:, 0])


@pytest.mark.parametrize("arch,L", [(dict(num_hidden_layers=2, vocab_size=2000), 48), ({}, 256)])
def test_cross_encoder_matches_transformers(gpu, arch, L):
    from audio_rag_amd.reranking.xlmr import CrossEncoderXLMR, build_reranker

    hf = build_reranker(seed=5, arch=dict(arch, attn_implementation="eager") if arch else
                        dict(attn_implementation="eager"))
    V = hf.config.vocab_size
    g = torch.Generator().manual_seed(4)
    n = 6
    ids = torch.randint(4, V, (n, L), generator=g)
    ids[:, 0] = 0
    mask = torch.ones(n, L, dtype=torch.long)
    for i in range(n):  # ragged pairs: <s> q </s></s> d </s> <pad>...
        ln = L - 9 * i
        ids[i, 16] = 2
        ids[i, 17] = 2
        ids[i, ln - 1] = 2
        ids[i, ln:] = 1
        mask[i, ln:] = 0
    ref = _hf_scores(hf, ids, mask)
    enc = CrossEncoderXLMR(hf, gpu)
    got = enc.forward(ids.int().to(gpu), mask.int().to(gpu)).cpu()
    torch.testing.assert_close(got, ref, rtol=0, atol=1e-3)


def test_reranker_rules_and_scores(gpu):
    from audio_rag_amd.config import RerankingConfig
    from audio_rag_amd.core import AudioChunk, RetrievalResult
    from audio_rag_amd.reranking.bge import BGEReranker

    rr = BGEReranker(RerankingConfig(), device=gpu, arch=dict(num_hidden_layers=2))
    res = [RetrievalResult(AudioChunk(text=f"chunk {i} text", start=i, end=i + 1), score=1 - i / 10,
                           source="c") for i in range(8)]
    out = rr.rerank("a query", res, top_k=3)
    assert len(out) == 3 and all(r.source is None for r in out)
    assert [r.score for r in out] == sorted([r.score for r in out], reverse=True)
    few = rr.rerank("a query", res[:3], top_k=5)  # bypass: sorted by retrieval score, no model
    assert [r.score for r in few] == [1.0, 0.9, 0.8] and few[0].source == "c"


def test_bge_m3_embedder_outputs(gpu):
    from audio_rag_amd.config import EmbeddingConfig
    from audio_rag_amd.embeddings.bge_m3 import BGEM3Embedder, build_bge_m3, lexical_weights

    arch = dict(num_hidden_layers=2)
    e = BGEM3Embedder(EmbeddingConfig(), device=gpu, arch=arch)
    r = e.embed_query("what does the lecturer say about gradient descent")
    d = np.array(r.dense)
    assert d.shape == (1024,) and abs(np.linalg.norm(d) - 1) < 2e-3
    assert np.array_equal(d.astype(np.float16).astype(np.float64), d)  # fp16-exact values
    assert r.sparse is not None and all(v > 0 for v in r.sparse.values)
    # against the fp32 CPU forward of the same seeded weights
    model, sparse = build_bge_m3(0, arch)
    ids = e.tokenizer.encode("what does the lecturer say about gradient descent")
    with torch.no_grad():
        h = model(input_ids=torch.tensor([ids])).last_hidden_state
        ref = torch.nn.functional.normalize(h[:, 0], dim=-1)[0].numpy()
        tw = torch.relu(sparse(h)).squeeze(-1)[0].tolist()
    assert np.dot(ref, d) > 0.999
    ref_lex = lexical_weights(tw, ids)
    got_lex = dict(zip(r.sparse.indices, r.sparse.values))
    # fp16 (GPU) vs fp32 (CPU): weights near the relu threshold may flip; compare the clear ones
    clear = [t for t, w in ref_lex.items() if w > 0.02]
    assert clear and all(t in got_lex for t in clear)
    assert all(ref_lex.get(t, 0.0) > 0 for t, w in got_lex.items() if w > 0.02)
    np.testing.assert_allclose([got_lex[t] for t in clear], [ref_lex[t] for t in clear],
                               rtol=2e-2, atol=2e-3)
    # keys keep first-occurrence order (FlagEmbedding dict order, bge.py:100)
    first = [t for t in dict.fromkeys(ids) if t in got_lex]
    assert r.sparse.indices == first


def _attention_ref(qkv, mask, H, dh):
    """Plain PyTorch fp32 eager attention (XLMRobertaSelfAttention) of the fp16 inputs."""
    n, L, _ = qkv.shape
    x = qkv.float().view(n, L, 3, H, dh).permute(2, 0, 3, 1, 4)
    q, k, v = x[0], x[1], x[2]
    add = (1 - mask.float())[:, None, None, :] * torch.finfo(torch.float32).min
    p = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(dh) + add, dim=-1)
    return (p @ v).permute(0, 2, 1, 3).reshape(n, L, H * dh)


@pytest.mark.parametrize("L", [1, 7, 33, 128, 200, 256, 512])
def test_attention_f16_matches_fp32_reference(gpu, L):
    """armi_enc_attention_f16 against fp32 eager attention of the same fp16 Q/K/V; tolerance
    3e-3 absolute + 1e-3 relative on O(1) outputs (P is rounded to fp16 before P.V, and the
    output itself is fp16: half an ulp is 4.9e-4 relative, 2e-3 at |o| = 4)."""
    g = torch.Generator().manual_seed(100 + L)
    n, H, dh = 3, 12, 64
    qkv = (torch.randn(n, L, 3 * H * dh, generator=g) * 1.5).half()
    mask = torch.ones(n, L, dtype=torch.int32)
    mask[1, max(1, L // 2):] = 0
    mask[2, 1:] = 0  # one key only
    ref = _attention_ref(qkv, mask, H, dh)
    Q, M = qkv.to(gpu).contiguous(), mask.to(gpu)
    out = torch.empty(n, L, H * dh, dtype=torch.float16, device=gpu)
    _call("armi_enc_attention_f16", Q.data_ptr(), M.data_ptr(), out.data_ptr(), n, L, H, dh,
          1 / math.sqrt(dh))
    torch.testing.assert_close(out.float().cpu(), ref, rtol=1e-3, atol=3e-3)


def test_attention_f16_peaked_scores(gpu):
    """Large, one-hot-like scores (the running max jumps late in the key sweep)."""
    n, L, H, dh = 2, 160, 12, 64
    g = torch.Generator().manual_seed(7)
    qkv = torch.randn(n, L, 3, H, dh, generator=g) * 0.1
    qkv[:, :, 1, :, :] *= 0.1
    qkv[:, 150, 1, :, :] = 4.0  # key 150 dominates every query
    qkv[:, :, 0, :, :] = qkv[:, :, 0, :, :].abs() + 0.5
    qkv = qkv.reshape(n, L, 3 * H * dh).half()
    mask = torch.ones(n, L, dtype=torch.int32)
    ref = _attention_ref(qkv, mask, H, dh)
    Q, M = qkv.to(gpu).contiguous(), mask.to(gpu)
    out = torch.empty(n, L, H * dh, dtype=torch.float16, device=gpu)
    _call("armi_enc_attention_f16", Q.data_ptr(), M.data_ptr(), out.data_ptr(), n, L, H, dh,
          1 / math.sqrt(dh))
    torch.testing.assert_close(out.float().cpu(), ref, rtol=1e-3, atol=3e-3)


@pytest.mark.parametrize("growth", [0.5, 9.0, 40.0])
def test_attention_f16_rising_scores(gpu, growth):
    """Scores that rise block after block (key j's K = (1 + growth * j / 32) * k0, queries
    aligned with k0), so the running maximum grows by less than, about and far more than the
    deferred-rescale threshold (2^8 in P) from one 32-key block to the next: every rescale
    decision (taken, skipped, first block) is exercised, ragged masks included."""
    n, L, H, dh = 3, 320, 12, 64
    g = torch.Generator().manual_seed(11)
    qkv = torch.randn(n, L, 3, H, dh, generator=g) * 0.3
    k0 = torch.randn(H, dh, generator=g)
    k0 = k0 / k0.norm(dim=-1, keepdim=True)
    ramp = 1 + growth * torch.arange(L, dtype=torch.float32) / 32
    qkv[:, :, 1] += (ramp[:, None, None] * k0[None]) * 2.0
    qkv[:, :, 0] += k0[None, None] * 2.5
    qkv = qkv.reshape(n, L, 3 * H * dh).half()
    mask = torch.ones(n, L, dtype=torch.int32)
    mask[1, 200:] = 0
    mask[2, 37:301] = 0
    ref = _attention_ref(qkv, mask, H, dh)
    Q, M = qkv.to(gpu).contiguous(), mask.to(gpu)
    out = torch.empty(n, L, H * dh, dtype=torch.float16, device=gpu)
    _call("armi_enc_attention_f16", Q.data_ptr(), M.data_ptr(), out.data_ptr(), n, L, H, dh,
          1 / math.sqrt(dh))
    torch.testing.assert_close(out.float().cpu(), ref, rtol=1e-3, atol=3e-3)


@pytest.mark.parametrize("L", [1, 7, 256, 300, 512])
def test_attention_cls_f16_matches_fp32_reference(gpu, L):
    """armi_enc_attention_cls_f16 (the <s> query only, the last layer's one consumer) against the
    position-0 row of fp32 eager attention; ragged masks incl. a single live key."""
    g = torch.Generator().manual_seed(300 + L)
    n, H, dh = 4, 12, 64
    qkv = (torch.randn(n, L, 3 * H * dh, generator=g) * 1.5).half()
    mask = torch.ones(n, L, dtype=torch.int32)
    mask[1, max(1, L // 2):] = 0
    mask[2, 1:] = 0
    ref = _attention_ref(qkv, mask, H, dh)[:, 0]
    Q, M = qkv.to(gpu).contiguous(), mask.to(gpu)
    out = torch.empty(n, H * dh, dtype=torch.float16, device=gpu)
    _call("armi_enc_attention_cls_f16", Q.data_ptr(), M.data_ptr(), out.data_ptr(), n, L, H, dh,
          1 / math.sqrt(dh))
    torch.testing.assert_close(out.float().cpu(), ref, rtol=0, atol=2e-3)


@pytest.mark.parametrize("width", [768, 1024, 640])  # vectorised (768, 1024) and generic kernels
def test_layernorm_f16_and_gelu_f16(gpu, width):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(300, width, generator=g).half()
    r = torch.randn(300, width, generator=g)
    w, b = torch.randn(width, generator=g), torch.randn(width, generator=g)
    ref = torch.nn.functional.layer_norm(x.float() + r, (width,), w, b, 1e-5)
    X, R, W, B = (t.to(gpu) for t in (x, r, w, b))
    out = torch.empty(300, width, device=gpu)
    out16 = torch.empty(300, width, dtype=torch.float16, device=gpu)
    _call("armi_enc_layernorm_residual_f16", X.data_ptr(), R.data_ptr(), W.data_ptr(),
          B.data_ptr(), out.data_ptr(), out16.data_ptr(), 300, width, 1e-5)
    torch.testing.assert_close(out.cpu(), ref, rtol=0, atol=2e-5)
    assert torch.equal(out16.cpu(), out.cpu().half())
    _call("armi_enc_layernorm_residual_f16", X.data_ptr(), None, W.data_ptr(), B.data_ptr(),
          out.data_ptr(), None, 300, width, 1e-5)
    torch.testing.assert_close(out.cpu(), torch.nn.functional.layer_norm(x.float(), (width,), w, b,
                                                                         1e-5), rtol=0, atol=2e-5)
    y = (torch.randn(64, 3072, generator=g) * 3).half()
    Y = y.to(gpu).contiguous()
    _call("armi_enc_gelu_f16", Y.data_ptr(), None, 64, 3072)
    torch.testing.assert_close(Y.cpu().float(), torch.nn.functional.gelu(y.float()), rtol=2e-3,
                               atol=2e-3)


@pytest.mark.parametrize("width", [768, 1024])
@pytest.mark.parametrize("rows", [1, 7, 300, 4097])  # odd counts: a half-wave with no row
def test_add_layernorm_f16(gpu, width, rows):
    """armi_enc_add_layernorm_f16: fp16 LayerNorm(x + res) of the all-fp16 residual stream (the
    reranker's post-attention / post-FFN norm, XLMRobertaSelfOutput / XLMRobertaOutput) against
    torch fp32 on the same fp16 inputs, within one fp16 rounding of the output."""
    g = torch.Generator().manual_seed(rows + width)
    x = torch.randn(rows, width, generator=g).half()
    r = (torch.randn(rows, width, generator=g) * 2).half()
    w, b = torch.randn(width, generator=g), torch.randn(width, generator=g)
    ref = torch.nn.functional.layer_norm(x.float() + r.float(), (width,), w, b, 1e-5)
    X, R, W, B = (t.to(gpu) for t in (x, r, w, b))
    out16 = torch.full((rows + 1, width), float("nan"), dtype=torch.float16, device=gpu)
    _call("armi_enc_add_layernorm_f16", X.data_ptr(), R.data_ptr(), W.data_ptr(), B.data_ptr(),
          out16.data_ptr(), rows, width, 1e-5)
    torch.cuda.synchronize()
    got = out16.cpu().float()
    torch.testing.assert_close(got[:rows], ref, rtol=2 ** -10, atol=1e-4)
    assert torch.isnan(got[rows]).all()  # nothing written past the last row


@pytest.mark.parametrize("L,residual", [(64, "fp16"), (256, "fp16"), (256, "fp32")])
def test_cross_encoder_fp16_within_1e3(gpu, L, residual):
    """north_star: rerank scores within 1e-3 on the fp16 path (fp16 GEMMs + fused fp16
    attention + fp32 LayerNorm statistics and residual stream) against transformers' fp32
    forward of the same seeded bge-reranker-base-shaped weights, ragged pairs included."""
    from audio_rag_amd.reranking.xlmr import CrossEncoderXLMR, build_reranker

    hf = build_reranker(seed=5, arch=dict(attn_implementation="eager"))
    g = torch.Generator().manual_seed(11)
    n = 8
    ids = torch.randint(4, hf.config.vocab_size, (n, L), generator=g)
    ids[:, 0] = 0
    mask = torch.ones(n, L, dtype=torch.long)
    for i in range(n):
        ln = L - 5 * i
        ids[i, 16] = 2
        ids[i, 17] = 2
        ids[i, ln - 1] = 2
        ids[i, ln:] = 1
        mask[i, ln:] = 0
    ref = _hf_scores(hf, ids, mask)
    enc = CrossEncoderXLMR(hf, gpu)
    enc.to_dtype(torch.float16, residual=residual)
    got = enc.forward(ids.int().to(gpu), mask.int().to(gpu)).cpu()
    err = (got - ref).abs().max().item()
    print(f"fp16 path max |score error| = {err:.2e} at L={L}, {residual} residual")
    (Path(__file__).resolve().parent.parent / "gpurun_out").mkdir(exist_ok=True)
    with open(Path(__file__).resolve().parent.parent / "gpurun_out" / "rerank_fp16_error.txt", "a") as f:
        f.write(f"L={L} n={n} residual={residual} max_abs_score_error={err:.3e}\n")
    torch.testing.assert_close(got, ref, rtol=0, atol=1e-3)


def test_cross_encoder_fp16_graph_replay_within_1e3(gpu):
    """The captured (HIP graph) fp16 forward, what BGEReranker and the configs[2] bench run:
    ragged pairs right-padded to the 32-token bucket (L = 121 -> 128) against transformers fp32
    (1e-3) and the eager forward of the same unpadded batch (GEMMs over other row counts may pick
    other library kernels: 1e-4); a second call of the same shape replays the cached graph."""
    from audio_rag_amd.reranking.xlmr import CrossEncoderXLMR, build_reranker

    hf = build_reranker(seed=5, arch=dict(attn_implementation="eager"))
    g = torch.Generator().manual_seed(12)
    n, L = 9, 121
    ids = torch.randint(4, hf.config.vocab_size, (n, L), generator=g)
    ids[:, 0] = 0
    mask = torch.ones(n, L, dtype=torch.long)
    for i in range(n):
        ln = L - 7 * i
        ids[i, 16] = 2
        ids[i, 17] = 2
        ids[i, ln - 1] = 2
        ids[i, ln:] = 1
        mask[i, ln:] = 0
    ref = _hf_scores(hf, ids, mask)
    enc = CrossEncoderXLMR(hf, gpu)
    enc.to_dtype(torch.float16)
    ids_d, mask_d = ids.int().to(gpu), mask.int().to(gpu)
    enc.use_graphs = False
    eager = enc.forward(ids_d, mask_d).cpu()
    enc.use_graphs = True
    graphed = enc.forward(ids_d, mask_d).cpu()
    assert list(enc._graphs) == [(enc._n_bucket(n), 128)]  # 9 pairs -> the 16-pair bucket
    again = enc.forward(ids_d.flip(0).contiguous(), mask_d.flip(0).contiguous()).cpu()
    assert len(enc._graphs) == 1
    torch.testing.assert_close(graphed, eager, rtol=0, atol=1e-4)
    torch.testing.assert_close(graphed, ref, rtol=0, atol=1e-3)
    torch.testing.assert_close(again, graphed.flip(0), rtol=0, atol=1e-5)


def test_cross_encoder_bf16_gemms_within_budget(gpu):
    """bf16 GEMM operands (fp32 accumulate, fp32 LN/softmax/GELU): measured distance to the fp32
    transformers forward at the full bge-reranker-base shape."""
    from audio_rag_amd.reranking.xlmr import CrossEncoderXLMR, build_reranker

    hf = build_reranker(seed=5, arch=dict(attn_implementation="eager"))
    g = torch.Generator().manual_seed(9)
    ids = torch.randint(4, hf.config.vocab_size, (8, 256), generator=g)
    ids[:, 0] = 0
    ids[:, 17] = 2
    ids[:, 18] = 2
    ids[:, -1] = 2
    mask = torch.ones_like(ids)
    ref = _hf_scores(hf, ids, mask)
    enc = CrossEncoderXLMR(hf, gpu)
    enc.to_dtype(torch.bfloat16)
    got = enc.forward(ids.int().to(gpu), mask.int().to(gpu)).cpu()
    err = (got - ref).abs().max().item()
    print(f"bf16 GEMM max |score error| = {err:.2e}")
    assert err < 1e-2


def test_bge_m3_query_graph_equals_eager(gpu):
    """The HIP-graph replay of a batch-1 query encode (padded to its length bucket) gives the
    eager forward's dense vector and lexical weights."""
    from audio_rag_amd.config import EmbeddingConfig
    from audio_rag_amd.embeddings.bge_m3 import BGEM3Embedder

    e = BGEM3Embedder(EmbeddingConfig(), device=gpu, arch=dict(num_hidden_layers=3))
    e.load()
    for text in ("short query", "what does the lecturer say about gradient descent and the "
                 "learning rate schedule in the third lecture of the course " * 2):
        seq = e.tokenizer.encode(text)
        dg, lg = e.encode_query_ids(seq)
        de, le = e.encode_ids([seq])
        torch.cuda.synchronize()
        cos = torch.nn.functional.cosine_similarity(dg.float(), de.float()).item()
        assert cos > 0.9999, cos
        clear = [t for t, w in le[0].items() if w > 0.02]
        assert all(t in lg[0] for t in clear)
        assert all(le[0].get(t, 0.0) > 0 for t, w in lg[0].items() if w > 0.02)
        np.testing.assert_allclose([lg[0][t] for t in clear], [le[0][t] for t in clear],
                                   rtol=5e-3, atol=1e-3)
    assert len(e._graphs) == 2  # one captured graph per length bucket used



def test_attention_f16_many_items_ragged(gpu):
    """Many sequences (840 (sequence, head) workgroups, more than the CUs) with a different ragged
    mask each (incl. a single live key and an all-live row), against fp32 eager attention."""
    g = torch.Generator().manual_seed(321)
    n, L, H, dh = 70, 200, 12, 64  # 840 items
    qkv = (torch.randn(n, L, 3 * H * dh, generator=g) * 1.5).half()
    lens = torch.randint(1, L + 1, (n,), generator=g)
    lens[0], lens[1] = L, 1
    mask = (torch.arange(L)[None, :] < lens[:, None]).to(torch.int32)
    ref = _attention_ref(qkv, mask, H, dh)
    Q, M = qkv.to(gpu).contiguous(), mask.to(gpu)
    out = torch.empty(n, L, H * dh, dtype=torch.float16, device=gpu)
    _call("armi_enc_attention_f16", Q.data_ptr(), M.data_ptr(), out.data_ptr(), n, L, H, dh,
          1 / math.sqrt(dh))
    torch.testing.assert_close(out.float().cpu(), ref, rtol=1e-3, atol=3e-3)
