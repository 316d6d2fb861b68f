"""fp16 XLM-R encoder forward on the armi kernels, for the batch-1 query encode of BGE-M3.

The same layer as transformers' XLMRobertaLayer (what BGEM3FlagModel runs,
src/audio_rag/embeddings/bge.py:42-157): embeddings + LayerNorm (armi_enc_embed_f16), then per
layer the fused Q|K|V projection, fused masked softmax attention (armi_enc_attention_f16), output
projection, add + LayerNorm (armi_enc_add_layernorm_f16), the intermediate dense with exact-erf
GELU fused into its GEMM and the output dense + add + LayerNorm; the residual stream is fp16 with fp32 LayerNorm statistics, as the cross-encoder's
default fp16 forward (reranking/xlmr.py). Outputs the dense vector (L2-normalised <s> row) and
the sparse head's token weights relu(Linear(d -> 1)(h)).

Six kernels per layer instead of the ~16 of the transformers forward: a captured query encode
is launch-bound (a 16-token query reads 0.6 GB of weights, 0.1 ms at HBM rate), so the kernel
count sets its latency. The four linears run on armi_enc_linear_small_f16 (the intermediate
dense with its GELU fused) at every row count, which makes the encode row-independent: the
batched query encode (BGEM3Embedder.embed_queries, QueryPipeline.query_batch) gives every query
the bits the batch-1 graph gives it, so query() and query_batch() rank identically.
"""

from __future__ import annotations

import math

import torch

from audio_rag_amd._armi import call, ptr, stream_handle


class XLMREncoderF16:
    """The query encoder. Built over the fp16 transformers model and sharing its tensors: the
    embedding tables are read in fp16 (armi_enc_embed_f16), and the model's query / key / value
    weights become views of the fused Q|K|V weight, so nothing is held twice (the fp32 word-table
    copy, 1 GB for BGE-M3, is gone since round 5)."""

    def __init__(self, hf_model, sparse_linear, device: torch.device):
        cfg = hf_model.config
        self.device = device
        self.d = cfg.hidden_size
        self.heads = cfg.num_attention_heads
        self.dh = self.d // self.heads
        if self.dh != 64 or self.d not in (768, 1024):
            raise ValueError("armi encoder kernels need head_dim 64 and width 768 or 1024")
        if next(hf_model.parameters()).dtype != torch.float16:
            raise ValueError("XLMREncoderF16 runs over the fp16 model")
        self.eps = float(cfg.layer_norm_eps)
        self.pad = cfg.pad_token_id
        f32 = lambda t: t.detach().float().contiguous()  # noqa: E731
        emb = hf_model.embeddings
        self.word = emb.word_embeddings.weight.detach()
        self.pos = emb.position_embeddings.weight.detach()
        self.type0 = emb.token_type_embeddings.weight.detach()[0]
        self.emb_ln = (f32(emb.LayerNorm.weight), f32(emb.LayerNorm.bias))
        self.layers = []
        d = self.d
        for layer in hf_model.encoder.layer:
            at = layer.attention.self
            with torch.no_grad():
                wqkv = torch.cat([at.query.weight, at.key.weight, at.value.weight]).contiguous()
                for j, lin in enumerate((at.query, at.key, at.value)):
                    lin.weight = torch.nn.Parameter(wqkv[j * d:(j + 1) * d], requires_grad=False)
            self.layers.append(dict(
                wqkv=wqkv,
                bqkv32=f32(torch.cat([at.query.bias, at.key.bias, at.value.bias])),
                wo=layer.attention.output.dense.weight.detach(),
                bo32=f32(layer.attention.output.dense.bias),
                ln1=(f32(layer.attention.output.LayerNorm.weight),
                     f32(layer.attention.output.LayerNorm.bias)),
                wi=layer.intermediate.dense.weight.detach(),
                bi32=f32(layer.intermediate.dense.bias),
                wo2=layer.output.dense.weight.detach(),
                bo232=f32(layer.output.dense.bias),
                ln2=(f32(layer.output.LayerNorm.weight), f32(layer.output.LayerNorm.bias)),
            ))
        self.sparse = None
        if sparse_linear is not None:
            # relu(Linear(d -> 1)) as a 16-column weight stream (columns 1..15 zero): the same
            # row-independent arithmetic as the encoder's linears
            w16 = torch.zeros((16, self.d), dtype=torch.float16, device=device)
            w16[0] = sparse_linear.weight.detach().to(device=device, dtype=torch.float16)[0]
            b16 = torch.zeros(16, dtype=torch.float32, device=device)
            b16[0] = sparse_linear.bias.detach().to(device=device, dtype=torch.float16).float()[0]
            self.sparse = dict(ws=w16, bs32=b16)

    def _lin(self, x: torch.Tensor, ly: dict, w: str, b: str, gelu: bool = False) -> torch.Tensor:
        """armi_enc_linear_small_f16 for every row count: each token row's result depends on
        that row alone, so a query's vector is the same bits alone and inside a batch (a query
        reads 0.6 GB of weights once per 32 token rows; queries are short)."""
        m = x.shape[0]
        n = ly[w].shape[0]
        out = torch.empty((m, n), dtype=torch.float16, device=self.device)
        call("armi_enc_linear_small_f16", ptr(x), ptr(ly[w]), ptr(ly[b + "32"]), ptr(out), m, n,
             ly[w].shape[1], 1 if gelu else 0, stream_handle())
        return out

    def forward(self, ids: torch.Tensor, mask: torch.Tensor):
        """ids, mask: int32 [n, L] on the device -> (dense fp16 [n, d] L2-normalised <s> rows,
        sparse token weights fp32 [n, L] or None). Row-independent: padding a sequence further
        (masked keys add exact zeros to the attention sums) or batching it with others leaves
        its outputs unchanged."""
        n, L = ids.shape
        d, H, dh = self.d, self.heads, self.dh
        s = stream_handle()
        rows = n * L
        h16 = torch.empty((rows, d), dtype=torch.float16, device=self.device)
        call("armi_enc_embed_f16", ptr(ids), ptr(self.word), ptr(self.pos), ptr(self.type0),
             ptr(self.emb_ln[0]), ptr(self.emb_ln[1]), ptr(h16), n, L, d, self.pad,
             self.word.shape[0], self.pos.shape[0], self.eps, s)
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
        # normalised one row at a time: the same [1, d] reduction for a query alone or in a batch
        cls = hid[:, 0]
        dense = torch.cat([torch.nn.functional.normalize(cls[i:i + 1], dim=-1) for i in range(n)])
        tw = None
        if self.sparse is not None:
            t16 = self._lin(h16, self.sparse, "ws", "bs")                    # [n*L, 16]
            tw = torch.relu(t16[:, 0]).float().view(n, L)
        return dense, tw
