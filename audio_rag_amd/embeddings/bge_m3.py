"""BGE-M3 query / chunk encoder on the MI355X (PyTorch-ROCm forward, as north_star allows).

Mirrors BGEM3Embedder (src/audio_rag/embeddings/bge.py:14-157) over FlagEmbedding's
BGEM3FlagModel (flagembedding >= 1.3.5, not installed):
  * model: XLM-RoBERTa-large (24 layers, d 1024, 16 heads, FFN 4096, vocab 250002, LN eps 1e-5)
    run in fp16 on the GPU (bge.py:54 use_fp16 on cuda)
  * dense  = L2-normalised hidden state of <s> (fp16 values, bge.py:149 .tolist())
  * sparse = relu(Linear(1024 -> 1)(hidden)) per token, max per token id, special tokens and
    weights <= 0 dropped, keys in first-occurrence order (_convert_sparse, bge.py:95-102)
Weights (load(), as BGEM3FlagModel(config.model) at bge.py:47-55): config.model naming a local
checkpoint directory or a cached hub snapshot loads its model.safetensors (or a weights-only
pytorch_model.bin), sparse_linear.pt and tokenizer.json (audio_rag_amd.checkpoints); otherwise
the encoder and the sparse head are initialised from EmbeddingConfig.seed and token ids come from
the stand-in tokenizer audio_rag_amd.text (BAAI/bge-m3 is not on disk here and cannot be
downloaded; documented in DESIGN.md). Token ids can also be passed directly (encode_ids).

Query encodes (embed_query, and embed_queries for QueryPipeline.query_batch) run on the armi
kernels (embeddings/xlmr_f16.py), whose arithmetic is row-independent: a query gets the same
vector alone and in a batch. embed() of corpus chunks runs transformers' fp16 forward.
"""

from __future__ import annotations

import gc
import logging

import torch

from audio_rag_amd.checkpoints import tokenizer_for
from audio_rag_amd.config.schema import EmbeddingConfig
from audio_rag_amd.core.base import BaseEmbedder, EmbeddingResult, SparseVector
from audio_rag_amd.core.exceptions import EmbeddingError
from audio_rag_amd.embeddings.base import EmbeddingsRegistry
from audio_rag_amd.text import SPECIAL_IDS, HashTokenizer, pad_batch
from audio_rag_amd.utils.decorators import require_loaded, timed

logger = logging.getLogger(__name__)

VRAM_ESTIMATE = 2.5  # GB (bge.py:11)

# XLM-RoBERTa-large as used by BAAI/bge-m3
BGE_M3_ARCH = dict(vocab_size=250002, hidden_size=1024, num_hidden_layers=24,
                   num_attention_heads=16, intermediate_size=4096, max_position_embeddings=8194,
                   layer_norm_eps=1e-5, pad_token_id=1, bos_token_id=0, eos_token_id=2,
                   type_vocab_size=1)


def build_bge_m3(seed: int, arch: dict | None = None):
    """Seeded random XLM-R encoder + sparse head (CPU, fp32)."""
    from transformers import XLMRobertaConfig, XLMRobertaModel

    cfg = XLMRobertaConfig(**{**BGE_M3_ARCH, **(arch or {})})
    g = torch.random.fork_rng()
    with g:
        torch.manual_seed(seed)
        model = XLMRobertaModel(cfg, add_pooling_layer=False)
        sparse_linear = torch.nn.Linear(cfg.hidden_size, 1)
    model.eval()
    return model, sparse_linear


def lexical_weights(token_weights: list[float], input_ids: list[int],
                    special_ids=SPECIAL_IDS) -> dict[int, float]:
    """FlagEmbedding's _process_token_weights: per token id the max weight, ids of special
    tokens (cls, eos, pad, unk) and weights <= 0 skipped, first-occurrence key order."""
    result: dict[int, float] = {}
    for w, idx in zip(token_weights, input_ids):
        if idx in special_ids or not w > 0:
            continue
        if w > result.get(idx, 0.0):
            result[idx] = w
    return result


def load_bge_m3(name: str, seed: int, arch: dict | None = None):
    """(encoder fp32 CPU, sparse head, tokenizer or None): the checkpoint config.model names when
    it is on disk (a directory or a cached hub snapshot), else the seeded stand-in."""
    from transformers import XLMRobertaModel

    from audio_rag_amd.checkpoints import load_pretrained, load_tokenizer, resolve_local

    path = resolve_local(name)
    if path is None:
        logger.warning(f"{name}: no local checkpoint; using seeded stand-in weights (seed {seed}) "
                       "and the stand-in tokenizer")
        model, sparse = build_bge_m3(seed, arch)
        return model, sparse, None
    model = load_pretrained(XLMRobertaModel, path, add_pooling_layer=False)
    sparse = torch.nn.Linear(model.config.hidden_size, 1)
    sp = path / "sparse_linear.pt"
    if sp.exists():
        sparse.load_state_dict(torch.load(str(sp), map_location="cpu", weights_only=True))
    else:
        logger.warning(f"{path}: no sparse_linear.pt; the sparse head is seeded (seed {seed})")
        with torch.random.fork_rng():
            torch.manual_seed(seed)
            sparse = torch.nn.Linear(model.config.hidden_size, 1)
    return model, sparse, load_tokenizer(path)


@EmbeddingsRegistry.register("bge-m3")
class BGEM3Embedder(BaseEmbedder):
    def __init__(self, config: EmbeddingConfig, device: torch.device | None = None,
                 arch: dict | None = None):
        self.config = config
        self._device = device or torch.device("cuda", 0)
        self._dimension = (arch or {}).get("hidden_size", BGE_M3_ARCH["hidden_size"])
        self._use_sparse = config.use_sparse
        self._arch = arch
        self._model = None
        self._sparse = None
        self._graphs: dict[int, tuple] = {}
        self._fast = None  # XLMREncoderF16 of the captured query encode (load())
        # the checkpoint's tokenizer.json when config.model is on disk, else the stand-in
        self.tokenizer = tokenizer_for(config.model) or HashTokenizer()
        logger.info(f"BGEM3Embedder initialized: model={config.model}, device={self._device}, "
                    f"sparse={self._use_sparse}")

    # The captured batch-1 query encode runs on the armi encoder kernels ("armi":
    # embeddings/xlmr_f16.py, 7 kernels per layer) or transformers' forward ("torch"). A class
    # attribute (tests set it per instance).
    query_kernels = "armi"

    def load(self) -> None:
        if self._model is not None:
            return
        try:
            logger.info(f"Loading {self.config.model} on {self._device}...")
            model, sparse, _ = load_bge_m3(self.config.model, self.config.seed, self._arch)
            self._model = model.to(self._device, dtype=torch.float16)
            self._sparse = sparse.to(self._device, dtype=torch.float16)
            self._dimension = model.config.hidden_size
        except Exception as e:
            raise EmbeddingError(f"Failed to load embedding model: {e}")
        self._fast = None
        # XLMREncoderF16 rebinds the model's query / key / value weights as views of its fused
        # Q|K|V tensor (one GEMM instead of three): the model must not be moved, cast or given a
        # new state dict in place afterwards (the two would silently stop sharing weights), so
        # the model and the encoder live and die together (unload() drops both; a new load()
        # rebuilds both from the same tensors)
        if self.query_kernels == "armi" and self._device.type == "cuda":
            from audio_rag_amd.embeddings.xlmr_f16 import XLMREncoderF16

            self._fast = XLMREncoderF16(self._model, self._sparse if self._use_sparse else None,
                                        self._device)
        logger.info(f"BGE-M3 loaded (dim={self._dimension}, sparse={self._use_sparse})")

    def unload(self) -> None:
        if self._model is None:
            return
        self._model = None
        self._sparse = None
        self._fast = None
        self._graphs.clear()
        gc.collect()
        torch.cuda.empty_cache()

    @property
    def is_loaded(self) -> bool:
        return self._model is not None

    @property
    def vram_required(self) -> float:
        return VRAM_ESTIMATE

    @property
    def dimension(self) -> int:
        return self._dimension

    @property
    def supports_sparse(self) -> bool:
        return self._use_sparse

    # ---------------------------------------------------------------------------- device

    @torch.inference_mode()
    def encode_ids(self, seqs: list[list[int]]) -> tuple[torch.Tensor, list[dict[int, float]] | None]:
        """Encodes token-id sequences; returns (dense fp16 [B, d] on the device, lexical
        weights per sequence or None)."""
        ids, mask = pad_batch(seqs)
        ids_t = torch.tensor(ids, dtype=torch.long, device=self._device)
        mask_t = torch.tensor(mask, dtype=torch.long, device=self._device)
        hidden = self._model(input_ids=ids_t, attention_mask=mask_t).last_hidden_state
        dense = torch.nn.functional.normalize(hidden[:, 0], dim=-1)
        lex = None
        if self._use_sparse:
            tw = torch.relu(self._sparse(hidden)).squeeze(-1).float().cpu().tolist()
            sp = self.tokenizer.special_ids
            lex = [lexical_weights(tw[i][: len(s)], s, sp) for i, s in enumerate(seqs)]
        return dense.contiguous(), lex

    # ------------------------------------------------------------- captured query encode

    GRAPH_BUCKETS = (16, 32, 64, 128, 256, 512)

    def _forward_static(self, ids_t: torch.Tensor, mask_t: torch.Tensor):
        if getattr(self, "_fast", None) is not None:
            return self._fast.forward(ids_t, mask_t)
        hidden = self._model(input_ids=ids_t, attention_mask=mask_t).last_hidden_state
        dense = torch.nn.functional.normalize(hidden[:, 0], dim=-1)
        tw = torch.relu(self._sparse(hidden)).squeeze(-1).float() if self._use_sparse else None
        return dense, tw

    def _graph_for(self, bucket: int):
        """(graph, static ids, static mask, static dense, static token weights) for a batch-1
        query padded to `bucket` tokens; captured on first use (torch.cuda.CUDAGraph = a HIP
        graph on ROCm), warmed up on a side stream first as capture requires."""
        g = self._graphs.get(bucket)
        if g is not None:
            return g
        idt = torch.int32 if getattr(self, "_fast", None) is not None else torch.long
        ids_t = torch.full((1, bucket), 1, dtype=idt, device=self._device)
        mask_t = torch.zeros((1, bucket), dtype=idt, device=self._device)
        ids_t[0, 0] = 0
        mask_t[0, 0] = 1
        side = torch.cuda.Stream(device=self._device)
        side.wait_stream(torch.cuda.current_stream(self._device))
        with torch.cuda.stream(side):
            for _ in range(2):
                self._forward_static(ids_t, mask_t)
        torch.cuda.current_stream(self._device).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            dense, tw = self._forward_static(ids_t, mask_t)
        g = (graph, ids_t, mask_t, dense, tw)
        self._graphs[bucket] = g
        return g

    @torch.inference_mode()
    def encode_query_ids(self, seq: list[int]) -> tuple[torch.Tensor, list[dict[int, float]] | None]:
        """encode_ids for one sequence through the captured graph of its length bucket (right
        padding with <pad> and a zero mask leaves the real tokens' outputs unchanged, as in any
        padded batch); sequences longer than the largest bucket run eagerly."""
        L = len(seq)
        bucket = next((b for b in self.GRAPH_BUCKETS if b >= L), None)
        if not self.config.query_graphs or bucket is None:
            return self.encode_query_batch([seq])
        graph, ids_t, mask_t, dense, tw = self._graph_for(bucket)
        ids_t.fill_(1)
        mask_t.zero_()
        ids_t[0, :L] = torch.tensor(seq, dtype=torch.long).to(self._device, non_blocking=True)
        mask_t[0, :L] = 1
        graph.replay()
        lex = None
        if self._use_sparse:
            lex = [lexical_weights(tw[0, :L].cpu().tolist(), seq, self.tokenizer.special_ids)]
        return dense.clone(), lex

    def _results(self, dense: torch.Tensor, lex) -> list[EmbeddingResult]:
        rows = dense.cpu().tolist()
        out = []
        for i, d in enumerate(rows):
            sparse = None
            if lex is not None:
                sparse = self._convert_sparse(lex[i])
            out.append(EmbeddingResult(dense=d, sparse=sparse))
        return out

    def _convert_sparse(self, sparse_dict: dict) -> SparseVector | None:
        """bge.py:95-102."""
        if not sparse_dict:
            return None
        return SparseVector(indices=[int(k) for k in sparse_dict.keys()],
                            values=[float(v) for v in sparse_dict.values()])

    # ----------------------------------------------------------------------------- API

    @timed
    @require_loaded
    def embed(self, texts: list[str]) -> list[EmbeddingResult]:
        if not texts:
            return []
        try:
            out = []
            bs = self.config.batch_size
            for a in range(0, len(texts), bs):
                seqs = [self.tokenizer.encode(t, self.config.max_length) for t in texts[a:a + bs]]
                out.extend(self._results(*self.encode_ids(seqs)))
            return out
        except Exception as e:
            raise EmbeddingError(f"Embedding generation failed: {e}")

    @require_loaded
    def embed_query(self, query: str) -> EmbeddingResult:
        try:
            seq = self.tokenizer.encode(query, self.config.max_length)
            return self._results(*self.encode_query_ids(seq))[0]
        except Exception as e:
            raise EmbeddingError(f"Query embedding failed: {e}")

    @require_loaded
    def embed_queries(self, queries: list[str]):
        """Batched query encode for the batched pipeline: (dense fp16 [B, d] device, lexical
        weights per query or None). On the armi query encoder (row-independent arithmetic), so
        every query gets exactly the vector and weights embed_query gives it."""
        seqs = [self.tokenizer.encode(q, self.config.max_length) for q in queries]
        return self.encode_query_batch(seqs)

    @torch.inference_mode()
    def encode_query_batch(self, seqs: list[list[int]]):
        """encode_ids for queries: the armi query encoder when loaded on the GPU (the same bits
        as encode_query_ids per sequence), else transformers' forward."""
        if getattr(self, "_fast", None) is None or not seqs:
            return self.encode_ids(seqs)
        ids, mask = pad_batch(seqs)
        ids_t = torch.tensor(ids, dtype=torch.int32, device=self._device)
        mask_t = torch.tensor(mask, dtype=torch.int32, device=self._device)
        dense, tw = self._fast.forward(ids_t, mask_t)
        lex = None
        if self._use_sparse:
            rows = tw.cpu().tolist()
            sp = self.tokenizer.special_ids
            lex = [lexical_weights(rows[i][: len(s)], s, sp) for i, s in enumerate(seqs)]
        return dense.contiguous(), lex
