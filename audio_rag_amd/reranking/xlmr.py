"""XLM-RoBERTa sequence-classification forward (the bge-reranker-base cross-encoder) on the
MI355X: the non-GEMM ops are libarmi kernels (armi_enc_*), the GEMMs go to hipBLASLt/rocBLAS
through torch.

Restates what sentence-transformers' CrossEncoder.predict runs for BGEReranker
(src/audio_rag/reranking/bge.py:51-55, 119-123): XLMRobertaForSequenceClassification with
num_labels = 1 (12 layers, d 768, 12 heads, FFN 3072, exact-erf GELU, LN eps 1e-5), head
dense -> tanh -> out_proj on <s>, then sigmoid. The fp32 path keeps ST's default dtype; the fp16
path (to_dtype(torch.float16)) runs fp16 GEMMs, the fused fp16 attention and an fp16 residual
stream with fp32 LayerNorm statistics: max |score error| 6.5e-5 - 9.6e-5 vs the fp32 forward
(budget 1e-3, tests/test_encoder_gpu.py).
"""

from __future__ import annotations

import logging
import math
from collections import OrderedDict

import torch

from audio_rag_amd._armi import call, ptr, stream_handle

logger = logging.getLogger(__name__)

# XLM-RoBERTa-base as used by BAAI/bge-reranker-base
RERANKER_ARCH = dict(vocab_size=250002, hidden_size=768, num_hidden_layers=12,
                     num_attention_heads=12, intermediate_size=3072, max_position_embeddings=514,
                     layer_norm_eps=1e-5, pad_token_id=1, bos_token_id=0, eos_token_id=2,
                     type_vocab_size=1, num_labels=1)


def build_reranker(seed: int, arch: dict | None = None):
    """Seeded random XLMRobertaForSequenceClassification (CPU, fp32, eager attention)."""
    from transformers import XLMRobertaConfig, XLMRobertaForSequenceClassification

    cfg = XLMRobertaConfig(**{**RERANKER_ARCH, **(arch or {})})
    with torch.random.fork_rng():
        torch.manual_seed(seed)
        model = XLMRobertaForSequenceClassification(cfg)
    model.eval()
    return model


class CrossEncoderXLMR:
    def __init__(self, hf_model, device: torch.device):
        cfg = hf_model.config
        self.device = device
        self.d = cfg.hidden_size
        self.heads = cfg.num_attention_heads
        self.dh = self.d // self.heads
        self.eps = float(cfg.layer_norm_eps)
        self.pad = cfg.pad_token_id
        sd = {k: v.detach().to(device=device, dtype=torch.float32).contiguous()
              for k, v in hf_model.state_dict().items()}
        e = "roberta.embeddings."
        self.word = sd[e + "word_embeddings.weight"]
        self.pos = sd[e + "position_embeddings.weight"]
        self.type0 = sd[e + "token_type_embeddings.weight"][0].contiguous()
        self.emb_ln = (sd[e + "LayerNorm.weight"], sd[e + "LayerNorm.bias"])
        self.layers = []
        for i in range(cfg.num_hidden_layers):
            p = f"roberta.encoder.layer.{i}."
            a = p + "attention.self."
            wqkv = torch.cat([sd[a + "query.weight"], sd[a + "key.weight"], sd[a + "value.weight"]])
            bqkv = torch.cat([sd[a + "query.bias"], sd[a + "key.bias"], sd[a + "value.bias"]])
            self.layers.append(dict(
                wqkv_t=wqkv.t().contiguous(), bqkv=bqkv,
                wo_t=sd[p + "attention.output.dense.weight"].t().contiguous(),
                bo=sd[p + "attention.output.dense.bias"],
                ln1=(sd[p + "attention.output.LayerNorm.weight"], sd[p + "attention.output.LayerNorm.bias"]),
                wi_t=sd[p + "intermediate.dense.weight"].t().contiguous(),
                bi=sd[p + "intermediate.dense.bias"],
                wo2_t=sd[p + "output.dense.weight"].t().contiguous(),
                bo2=sd[p + "output.dense.bias"],
                ln2=(sd[p + "output.LayerNorm.weight"], sd[p + "output.LayerNorm.bias"]),
            ))
        self.gemm_dtype = torch.float32
        self.residual = "fp32"
        # dense weight transposed ([in][out]): armi_enc_cls_head_sigmoid reads it coalesced
        self.head = (sd["classifier.dense.weight"].t().contiguous(), sd["classifier.dense.bias"],
                     sd["classifier.out_proj.weight"].reshape(-1).contiguous(),
                     sd["classifier.out_proj.bias"])

    def to_dtype(self, dtype: torch.dtype, residual: str = "fp16") -> None:
        """GEMM operand dtype, fp32 accumulate.
        fp32 / bf16: LayerNorm / softmax / GELU / head stay fp32 in the armi kernels.
        fp16: the fp16 forward (_forward_f16): fp16 GEMM outputs, fused fp16 attention
        (armi_enc_attention_f16), LayerNorm statistics in fp32; the residual stream is fp16
        (residual="fp16", the default: half the LayerNorm traffic) or fp32 ("fp32")."""
        if residual not in ("fp16", "fp32"):
            raise ValueError("residual must be 'fp16' or 'fp32'")
        self.residual = residual
        self.gemm_dtype = dtype
        if dtype == torch.float16:
            # fp16 embedding tables: the fp16 forward embeds straight to fp16 (armi_enc_embed_f16)
            self.word16, self.pos16, self.type16 = (t.half() for t in (self.word, self.pos,
                                                                       self.type0))
        for ly in self.layers:
            for name in ("wqkv_t", "wo_t", "wi_t", "wo2_t"):
                ly[name + "_g"] = ly[name].to(dtype)
            if dtype == torch.float16:
                # nn.Linear layout [out, in] for F.linear and the armi GEMMs
                for name in ("wqkv_t", "wo_t", "wi_t", "wo2_t"):
                    ly[name[:-2] + "_h"] = ly[name].t().contiguous().half()
                for name in ("bqkv", "bo", "bi", "bo2"):
                    ly[name + "_h"] = ly[name].half()

    def _forward_f16(self, ids: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        n, L = ids.shape
        d, H, dh = self.d, self.heads, self.dh
        s = stream_handle()
        rows = n * L
        lin = torch.nn.functional.linear
        if self.residual == "fp16":
            h16 = torch.empty((rows, d), dtype=torch.float16, device=self.device)
            call("armi_enc_embed_f16", ptr(ids), ptr(self.word16), ptr(self.pos16),
                 ptr(self.type16), ptr(self.emb_ln[0]), ptr(self.emb_ln[1]), ptr(h16), n, L, d,
                 self.pad, self.word.shape[0], self.pos.shape[0], self.eps, s)
            return self._layers_f16_residual(h16, mask, n, L)
        h = torch.empty((rows, d), dtype=torch.float32, device=self.device)
        call("armi_enc_embed", ptr(ids), ptr(self.word), ptr(self.pos), ptr(self.type0),
             ptr(self.emb_ln[0]), ptr(self.emb_ln[1]), ptr(h), n, L, d, self.pad,
             self.word.shape[0], self.pos.shape[0], self.eps, s)
        h16 = h.half()
        scale = 1.0 / math.sqrt(dh)
        for ly in self.layers:
            qkv = lin(h16, ly["wqkv_h"], ly["bqkv_h"])                     # [n*L, 3d] fp16
            ctx = torch.empty((rows, d), dtype=torch.float16, device=self.device)
            call("armi_enc_attention_f16", ptr(qkv), ptr(mask), ptr(ctx), n, L, H, dh, scale, s)
            attn = lin(ctx, ly["wo_h"], ly["bo_h"])
            h1 = torch.empty_like(h)
            h1_16 = torch.empty_like(h16)
            call("armi_enc_layernorm_residual_f16", ptr(attn), ptr(h), ptr(ly["ln1"][0]),
                 ptr(ly["ln1"][1]), ptr(h1), ptr(h1_16), rows, d, self.eps, s)
            inter = lin(h1_16, ly["wi_h"], ly["bi_h"])                      # [n*L, 4d] fp16
            call("armi_enc_gelu_f16", ptr(inter), None, rows, inter.shape[1], s)
            out = lin(inter, ly["wo2_h"], ly["bo2_h"])
            h = torch.empty_like(h1)
            h16 = torch.empty_like(h1_16)
            call("armi_enc_layernorm_residual_f16", ptr(out), ptr(h1), ptr(ly["ln2"][0]),
                 ptr(ly["ln2"][1]), ptr(h), ptr(h16), rows, d, self.eps, s)
        probs = torch.empty(n, dtype=torch.float32, device=self.device)
        call("armi_enc_cls_head_sigmoid", ptr(h), ptr(self.head[0]), ptr(self.head[1]),
             ptr(self.head[2]), ptr(self.head[3]), ptr(probs), n, L, d, s)
        return probs

    # Linear layers of the fp16 forward: "armi" = armi_enc_linear_f16 (hand-written gfx950 GEMM,
    # bias / bias + exact-erf GELU fused into the epilogue: no separate GELU pass), "torch" = torch's
    # hipBLASLt linear + armi_enc_gelu_f16. "mixed" (default) = armi for the FFN-up GEMM only, whose
    # fused GELU saves the activation round trip (2.14 ms vs 2.22 + 0.55 ms per layer at 1,280 x
    # 256 tokens), hipBLASLt for the other three, where it is 18-28 % faster than the hand-written
    # GEMM (profiles/r03c_gemm.log). A class attribute (tests set it per instance).
    gemm_impl = "mixed"

    def _lin(self, x: torch.Tensor, ly: dict, name: str, gelu: bool = False) -> torch.Tensor:
        """y = x . W^T + b (+ exact GELU) for weight `name` of layer ly, fp16 in / out."""
        w, b = ly[name + "_h"], ly[{"wqkv": "bqkv", "wo": "bo", "wi": "bi", "wo2": "bo2"}[name]]
        n, k = w.shape
        own = self.gemm_impl == "armi" or (self.gemm_impl == "mixed" and gelu)
        if own and n % 256 == 0 and k % 64 == 0 and k >= 128:
            out = torch.empty((x.shape[0], n), dtype=torch.float16, device=self.device)
            call("armi_enc_linear_f16", ptr(x), ptr(w), ptr(b), ptr(out), x.shape[0], n, k,
                 1 if gelu else 0, stream_handle())
            return out
        y = torch.nn.functional.linear(x, w, ly[{"wqkv": "bqkv", "wo": "bo", "wi": "bi",
                                                 "wo2": "bo2"}[name] + "_h"])
        if gelu:
            call("armi_enc_gelu_f16", ptr(y), None, y.shape[0], y.shape[1], stream_handle())
        return y

    def _layers_f16_residual(self, h16: torch.Tensor, mask: torch.Tensor, n: int,
                             L: int) -> torch.Tensor:
        """Encoder layers with an all-fp16 residual stream (armi_enc_add_layernorm_f16: fp16 in
        and out, fp32 statistics), then the classification head on the fp32 <s> rows."""
        for _ in self._layer_ops(h16, mask, n, L):
            pass
        return self._result

    def _layer_ops(self, h16: torch.Tensor, mask: torch.Tensor, n: int, L: int):
        """Generator over the launches of _layers_f16_residual on the caller's current stream
        (one yield per kernel); returns the [n] probabilities (also left in self._result)."""
        d, H, dh = self.d, self.heads, self.dh
        s = stream_handle()
        rows = n * L
        scale = 1.0 / math.sqrt(dh)
        last = len(self.layers) - 1
        for i, ly in enumerate(self.layers):
            qkv = self._lin(h16, ly, "wqkv")
            yield
            if i == last:
                # The head reads only the <s> row of the last layer's output, and every op after
                # the attention is row-wise: the last layer runs its attention for the <s> query
                # alone (over all keys) and its output projection, LayerNorms and FFN on those n
                # rows, not on n * L. The <s> rows come out the same as in the full layer.
                ctx = torch.empty((n, d), dtype=torch.float16, device=self.device)
                call("armi_enc_attention_cls_f16", ptr(qkv), ptr(mask), ptr(ctx), n, L, H, dh,
                     scale, s)
                h16, rows = h16.view(n, L, d)[:, 0].contiguous(), n
            else:
                ctx = torch.empty((rows, d), dtype=torch.float16, device=self.device)
                call("armi_enc_attention_f16", ptr(qkv), ptr(mask), ptr(ctx), n, L, H, dh, scale,
                     s)
            del qkv
            yield
            attn = self._lin(ctx, ly, "wo")
            yield
            h1 = torch.empty_like(h16)
            call("armi_enc_add_layernorm_f16", ptr(attn), ptr(h16), ptr(ly["ln1"][0]),
                 ptr(ly["ln1"][1]), ptr(h1), rows, d, self.eps, s)
            del attn
            yield
            inter = self._lin(h1, ly, "wi", gelu=True)  # exact-erf GELU in the epilogue
            yield
            out = self._lin(inter, ly, "wo2")
            del inter
            yield
            h16 = torch.empty_like(h1)
            call("armi_enc_add_layernorm_f16", ptr(out), ptr(h1), ptr(ly["ln2"][0]),
                 ptr(ly["ln2"][1]), ptr(h16), rows, d, self.eps, s)
            del out
            yield
        cls = h16.float()  # [n, d]: the last layer's <s> rows
        probs = torch.empty(n, dtype=torch.float32, device=self.device)
        call("armi_enc_cls_head_sigmoid", ptr(cls), ptr(self.head[0]), ptr(self.head[1]),
             ptr(self.head[2]), ptr(self.head[3]), ptr(probs), n, 1, d, s)
        self._result = probs
        return probs

    def flops(self, n: int, L: int) -> float:
        """Matmul FLOPs one forward over n sequences of length L computes (projections, FFN,
        QK^T and PV; the fused attention recomputes QK^T once more, not counted). The default
        fp16 forward's last layer computes only the <s> rows after its QKV projection."""
        d, ff, layers = self.d, self.layers[0]["wi_t"].shape[1], len(self.layers)
        per_tok = 2 * (4 * d * d + 2 * d * ff)
        attn = 2 * 2 * L * L * d
        full = float(layers * (n * L * per_tok + n * attn))
        if self.gemm_dtype != torch.float16 or self.residual != "fp16":
            return full
        last = n * L * 2 * 3 * d * d + n * 2 * 2 * L * d + n * 2 * (d * d + 2 * d * ff)
        return float((layers - 1) * (n * L * per_tok + n * attn) + last)

    def _mm(self, x: torch.Tensor, ly: dict, name: str, bias: torch.Tensor | None) -> torch.Tensor:
        if self.gemm_dtype == torch.float32:
            w = ly[name]
            return torch.addmm(bias, x, w) if bias is not None else torch.mm(x, w)
        y = torch.mm(x.to(self.gemm_dtype), ly[name + "_g"]).float()
        return y.add_(bias) if bias is not None else y

    # Captured forwards (HIP graphs through torch.cuda.CUDAGraph), keyed by (n, L bucket): one
    # replay issues every kernel of the forward with no host work between them (the eager
    # forward's ~130 launches, hipBLASLt's per-call argument uploads and allocator calls
    # otherwise leave the GPU idle between kernels). Sequences are right-padded with <pad>
    # (mask 0) to the bucket: the real tokens' outputs, and so the <s> row the head reads, are
    # those of the unpadded batch.
    # The pair count is bucketed too (multiples of 8 up to 128 pairs, of 64 above; the extra rows
    # are <s>-only sequences whose scores are dropped), and every capture allocates from one
    # shared memory pool (replays are serial on one stream and each result is copied out at
    # once, so one graph's dead activations may back another's): variable candidate counts no
    # longer pin one activation-sized pool per (n, L).
    use_graphs = True
    GRAPH_L_STEP = 32
    MAX_GRAPHS = 8

    @staticmethod
    def _n_bucket(n: int) -> int:
        step = 8 if n <= 128 else 64
        return -(-n // step) * step

    def _graph_for(self, n: int, L: int):
        key = (n, L)
        g = self._graphs.get(key) if hasattr(self, "_graphs") else None
        if g is not None:
            self._graphs.move_to_end(key)
            return g
        if not hasattr(self, "_graphs"):
            self._graphs = OrderedDict()
        ids_t = torch.full((n, L), self.pad, dtype=torch.int32, device=self.device)
        mask_t = torch.zeros((n, L), dtype=torch.int32, device=self.device)
        ids_t[:, 0] = 0
        mask_t[:, 0] = 1
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(2):  # warm-up: library handles, kernel attributes, allocator blocks
                self._forward_eager(ids_t, mask_t)
        torch.cuda.current_stream(self.device).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        if getattr(self, "_pool", None) is None:
            self._pool = torch.cuda.graph_pool_handle()
        with torch.cuda.graph(graph, pool=self._pool):
            probs = self._forward_eager(ids_t, mask_t)
        g = (graph, ids_t, mask_t, probs)
        self._graphs[key] = g
        while len(self._graphs) > self.MAX_GRAPHS:
            self._graphs.popitem(last=False)
        return g

    def _forward_graphed(self, ids: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        n, L = ids.shape
        Lb = min(-(-L // self.GRAPH_L_STEP) * self.GRAPH_L_STEP, self.pos.shape[0] - self.pad - 1)
        if Lb < L:
            return self._forward_eager(ids, mask)
        nb = self._n_bucket(n)
        graph, ids_t, mask_t, probs = self._graph_for(nb, Lb)
        if Lb > L:
            ids_t[:n, L:].fill_(self.pad)
            mask_t[:n, L:].zero_()
        ids_t[:n, :L].copy_(ids)
        mask_t[:n, :L].copy_(mask)
        if nb > n:  # padding pairs: <s> alone (their scores are dropped)
            ids_t[n:].fill_(self.pad)
            mask_t[n:].zero_()
            ids_t[n:, 0] = 0
            mask_t[n:, 0] = 1
        graph.replay()
        return probs[:n].clone()

    @torch.inference_mode()
    def forward(self, ids: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        """ids, mask: int32 [n, L] on the device -> sigmoid scores float32 [n]."""
        if self.use_graphs and self.gemm_dtype == torch.float16 and self.residual == "fp16":
            try:
                return self._forward_graphed(ids, mask)
            except RuntimeError as e:  # capture refused: the same kernels, launched eagerly
                logger.warning(f"cross-encoder graph capture failed ({e}); running eagerly")
                self.use_graphs = False
        return self._forward_eager(ids, mask)

    def _forward_eager(self, ids: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        if self.gemm_dtype == torch.float16:
            return self._forward_f16(ids, mask)
        n, L = ids.shape
        d, H, dh = self.d, self.heads, self.dh
        s = stream_handle()
        h = torch.empty((n * L, d), dtype=torch.float32, device=self.device)
        call("armi_enc_embed", ptr(ids), ptr(self.word), ptr(self.pos), ptr(self.type0),
             ptr(self.emb_ln[0]), ptr(self.emb_ln[1]), ptr(h), n, L, d, self.pad,
             self.word.shape[0], self.pos.shape[0], self.eps, s)
        scale = 1.0 / math.sqrt(dh)
        for ly in self.layers:
            qkv = self._mm(h, ly, "wqkv_t", ly["bqkv"])                     # [n*L, 3d]
            qkv = qkv.view(n, L, 3, H, dh).permute(2, 0, 3, 1, 4)          # [3, n, H, L, dh]
            q, k, v = qkv[0], qkv[1], qkv[2]
            if self.gemm_dtype == torch.float32:
                scores = torch.matmul(q, k.transpose(-1, -2)).contiguous()  # [n, H, L, L]
            else:
                scores = torch.matmul(q.to(self.gemm_dtype),
                                      k.to(self.gemm_dtype).transpose(-1, -2)).float().contiguous()
            call("armi_enc_masked_softmax", ptr(scores), ptr(mask), n, H, L, scale, s)
            if self.gemm_dtype == torch.float32:
                ctx = torch.matmul(scores, v)
            else:
                ctx = torch.matmul(scores.to(self.gemm_dtype), v.to(self.gemm_dtype)).float()
            ctx = ctx.permute(0, 2, 1, 3).reshape(n * L, d)
            attn = self._mm(ctx, ly, "wo_t", ly["bo"])
            h1 = torch.empty_like(h)
            call("armi_enc_layernorm_residual", ptr(attn), ptr(h), ptr(ly["ln1"][0]),
                 ptr(ly["ln1"][1]), ptr(h1), n * L, d, self.eps, s)
            inter = self._mm(h1, ly, "wi_t", None)
            call("armi_enc_bias_gelu", ptr(inter), ptr(ly["bi"]), n * L, inter.shape[1], s)
            out = self._mm(inter, ly, "wo2_t", ly["bo2"])
            h = torch.empty_like(h)
            call("armi_enc_layernorm_residual", ptr(out), ptr(h1), ptr(ly["ln2"][0]),
                 ptr(ly["ln2"][1]), ptr(h), n * L, d, self.eps, s)
        probs = torch.empty(n, dtype=torch.float32, device=self.device)
        call("armi_enc_cls_head_sigmoid", ptr(h), ptr(self.head[0]), ptr(self.head[1]),
             ptr(self.head[2]), ptr(self.head[3]), ptr(probs), n, L, d, s)
        return probs
