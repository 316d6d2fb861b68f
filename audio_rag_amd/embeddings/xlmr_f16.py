"""fp16 XLM-R encoder forward on the armi kernels, for the batch-1 query encode of BGE-M3.

The same layer as transformers' XLMRobertaLayer (what BGEM3FlagModel runs,
src/audio_rag/embeddings/bge.py:42-157): embeddings + LayerNorm (armi_enc_embed), then per layer
the fused Q|K|V projection (hipBLASLt through F.linear), fused masked softmax attention
(armi_enc_attention_f16), output projection, add + LayerNorm (armi_enc_add_layernorm_f16), the
intermediate dense with exact-erf GELU (armi_enc_gelu_f16) and the output dense + add +
LayerNorm; the residual stream is fp16 with fp32 LayerNorm statistics, as the cross-encoder's
default fp16 forward (reranking/xlmr.py). Outputs the dense vector (L2-normalised <s> row) and
the sparse head's token weights relu(Linear(d -> 1)(h)).

Seven kernels per layer instead of the ~16 of the transformers forward: a captured query encode
is launch-bound (a 16-token query reads 0.6 GB of weights, 0.1 ms at HBM rate), so the kernel
count sets its latency. Up to 32 token rows the four linears run on armi_enc_linear_small_f16
(the intermediate dense with its GELU fused: six kernels per layer).
"""

from __future__ import annotations

import math

import torch

from audio_rag_amd._armi import call, ptr, stream_handle


class XLMREncoderF16:
    def __init__(self, hf_model, sparse_linear, device: torch.device):
        cfg = hf_model.config
        self.device = device
        self.d = cfg.hidden_size
        self.heads = cfg.num_attention_heads
        self.dh = self.d // self.heads
        if self.dh != 64 or self.d not in (768, 1024):
            raise ValueError("armi encoder kernels need head_dim 64 and width 768 or 1024")
        self.eps = float(cfg.layer_norm_eps)
        self.pad = cfg.pad_token_id
        sd = {k: v.detach().to(device=device) for k, v in hf_model.state_dict().items()}
        f32 = lambda t: t.float().contiguous()  # noqa: E731
        f16 = lambda t: t.half().contiguous()  # noqa: E731
        self.word = f32(sd["embeddings.word_embeddings.weight"])
        self.pos = f32(sd["embeddings.position_embeddings.weight"])
        self.type0 = f32(sd["embeddings.token_type_embeddings.weight"][0])
        self.emb_ln = (f32(sd["embeddings.LayerNorm.weight"]), f32(sd["embeddings.LayerNorm.bias"]))
        self.layers = []
        for i in range(cfg.num_hidden_layers):
            p = f"encoder.layer.{i}."
            a = p + "attention.self."
            self.layers.append(dict(
                wqkv=f16(torch.cat([sd[a + "query.weight"], sd[a + "key.weight"],
                                    sd[a + "value.weight"]])),
                bqkv32=f32(torch.cat([sd[a + "query.bias"], sd[a + "key.bias"],
                                      sd[a + "value.bias"]])),
                bo32=f32(sd[p + "attention.output.dense.bias"]),
                bi32=f32(sd[p + "intermediate.dense.bias"]),
                bo232=f32(sd[p + "output.dense.bias"]),
                bqkv=f16(torch.cat([sd[a + "query.bias"], sd[a + "key.bias"],
                                    sd[a + "value.bias"]])),
                wo=f16(sd[p + "attention.output.dense.weight"]),
                bo=f16(sd[p + "attention.output.dense.bias"]),
                ln1=(f32(sd[p + "attention.output.LayerNorm.weight"]),
                     f32(sd[p + "attention.output.LayerNorm.bias"])),
                wi=f16(sd[p + "intermediate.dense.weight"]),
                bi=f16(sd[p + "intermediate.dense.bias"]),
                wo2=f16(sd[p + "output.dense.weight"]),
                bo2=f16(sd[p + "output.dense.bias"]),
                ln2=(f32(sd[p + "output.LayerNorm.weight"]), f32(sd[p + "output.LayerNorm.bias"])),
            ))
        self.sparse = None
        if sparse_linear is not None:
            self.sparse = (f16(sparse_linear.weight.detach().to(device)),
                           f16(sparse_linear.bias.detach().to(device)))

    # token rows up to which the linears run on armi_enc_linear_small_f16 (a weight stream with
    # the GELU fused) instead of hipBLASLt
    SMALL_M = 32

    def _lin(self, x: torch.Tensor, ly: dict, w: str, b: str, gelu: bool = False) -> torch.Tensor:
        m = x.shape[0]
        if m <= self.SMALL_M:
            n = ly[w].shape[0]
            out = torch.empty((m, n), dtype=torch.float16, device=self.device)
            call("armi_enc_linear_small_f16", ptr(x), ptr(ly[w]), ptr(ly[b + "32"]), ptr(out), m,
                 n, ly[w].shape[1], 1 if gelu else 0, stream_handle())
            return out
        y = torch.nn.functional.linear(x, ly[w], ly[b])
        if gelu:
            call("armi_enc_gelu_f16", ptr(y), None, y.shape[0], y.shape[1], stream_handle())
        return y

    def forward(self, ids: torch.Tensor, mask: torch.Tensor):
        """ids, mask: int32 [n, L] on the device -> (dense fp16 [n, d] L2-normalised <s> rows,
        sparse token weights fp32 [n, L] or None)."""
        n, L = ids.shape
        d, H, dh = self.d, self.heads, self.dh
        s = stream_handle()
        rows = n * L
        lin = torch.nn.functional.linear
        h = torch.empty((rows, d), dtype=torch.float32, device=self.device)
        call("armi_enc_embed", ptr(ids), ptr(self.word), ptr(self.pos), ptr(self.type0),
             ptr(self.emb_ln[0]), ptr(self.emb_ln[1]), ptr(h), n, L, d, self.pad,
             self.word.shape[0], self.pos.shape[0], self.eps, s)
        h16 = h.half()
        scale = 1.0 / math.sqrt(dh)
        for ly in self.layers:
            qkv = self._lin(h16, ly, "wqkv", "bqkv")                         # [n*L, 3d]
            ctx = torch.empty((rows, d), dtype=torch.float16, device=self.device)
            call("armi_enc_attention_f16", ptr(qkv), ptr(mask), ptr(ctx), n, L, H, dh, scale, s)
            attn = self._lin(ctx, ly, "wo", "bo")
            h1 = torch.empty_like(h16)
            call("armi_enc_add_layernorm_f16", ptr(attn), ptr(h16), ptr(ly["ln1"][0]),
                 ptr(ly["ln1"][1]), ptr(h1), rows, d, self.eps, s)
            inter = self._lin(h1, ly, "wi", "bi", gelu=True)                 # [n*L, 4d]
            out = self._lin(inter, ly, "wo2", "bo2")
            h16 = torch.empty_like(h1)
            call("armi_enc_add_layernorm_f16", ptr(out), ptr(h1), ptr(ly["ln2"][0]),
                 ptr(ly["ln2"][1]), ptr(h16), rows, d, self.eps, s)
        hid = h16.view(n, L, d)
        dense = torch.nn.functional.normalize(hid[:, 0], dim=-1)
        tw = None
        if self.sparse is not None:
            tw = torch.relu(lin(hid, self.sparse[0], self.sparse[1])).squeeze(-1).float()
        return dense, tw
