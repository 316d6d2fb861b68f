"""BGEReranker on the MI355X (mirrors src/audio_rag/reranking/bge.py:14-147).

rerank() keeps the reference's rules exactly:
  * empty input -> returned as is; len(results) <= top_k -> sorted by retrieval score, no model
    (bge.py:104-109)
  * otherwise score every (query, chunk.text) pair with the cross-encoder (sigmoid of the
    logit), build fresh RetrievalResult(chunk, score) with source=None (bge.py:116-131),
    stable sort descending, keep top_k (bge.py:134, 141)
  * any failure -> warning + the retrieval results sorted by score, top_k (bge.py:143-147)
Weights (load(), as CrossEncoder(config.model, max_length=512) at bge.py:50-55): config.model
naming a local checkpoint directory or a cached hub snapshot loads its model.safetensors (or a
weights-only pytorch_model.bin) and tokenizer.json (audio_rag_amd.checkpoints); otherwise
(BAAI/bge-reranker-base is not on disk here) the model is initialised from RerankingConfig.seed
and token ids come from the stand-in tokenizer audio_rag_amd.text. score_ids() takes ids directly.
"""

from __future__ import annotations

import logging

import torch

from audio_rag_amd.config.schema import RerankingConfig
from audio_rag_amd.core.base import RetrievalResult
from audio_rag_amd.core.exceptions import RerankingError
from audio_rag_amd.reranking.base import BaseReranker, RerankerRegistry
from audio_rag_amd.checkpoints import tokenizer_for
from audio_rag_amd.reranking.xlmr import CrossEncoderXLMR, build_reranker
from audio_rag_amd.text import HashTokenizer, pad_batch, pair_ids

logger = logging.getLogger(__name__)


def load_reranker(name: str, seed: int, arch: dict | None = None):
    """(XLMRobertaForSequenceClassification fp32 CPU, tokenizer or None): the checkpoint
    config.model names when it is on disk, else the seeded stand-in."""
    from transformers import XLMRobertaForSequenceClassification

    from audio_rag_amd.checkpoints import load_pretrained, load_tokenizer, resolve_local

    path = resolve_local(name)
    if path is None:
        logger.warning(f"{name}: no local checkpoint; using seeded stand-in weights (seed {seed}) "
                       "and the stand-in tokenizer")
        return build_reranker(seed, arch), None
    hf = load_pretrained(XLMRobertaForSequenceClassification, path)
    if hf.config.num_labels != 1:
        raise ValueError(f"{path}: a cross-encoder has one output logit, not {hf.config.num_labels}")
    return hf, load_tokenizer(path)


@RerankerRegistry.register("bge-reranker")
class BGEReranker(BaseReranker):
    MODEL_VRAM = {"BAAI/bge-reranker-base": 0.5, "BAAI/bge-reranker-large": 1.2,
                  "BAAI/bge-reranker-v2-m3": 1.5}

    def __init__(self, config: RerankingConfig, device: torch.device | None = None,
                 arch: dict | None = None):
        super().__init__(config)
        self._device = device or torch.device("cuda", 0)
        self._arch = arch
        self._model: CrossEncoderXLMR | None = None
        # the checkpoint's tokenizer.json when config.model is on disk (known before load(): a
        # lazy load() inside rerank() must not change how that call tokenised), else the stand-in
        self.tokenizer = tokenizer_for(config.model) or HashTokenizer()

    @property
    def vram_required(self) -> float:
        return self.MODEL_VRAM.get(self.config.model, 1.0)

    def load(self) -> None:
        if self._is_loaded:
            return
        try:
            logger.info(f"Loading reranker {self.config.model} on {self._device}")
            hf, _ = load_reranker(self.config.model, self.config.seed, self._arch)
            self._model = CrossEncoderXLMR(hf, self._device)
            if self.config.dtype == "fp16":
                self._model.to_dtype(torch.float16)
            self._is_loaded = True
        except Exception as e:
            raise RerankingError(f"Failed to load reranker: {e}") from e

    def unload(self) -> None:
        self._model = None
        self._is_loaded = False
        torch.cuda.empty_cache()

    def score_ids(self, pairs: list[list[int]]) -> torch.Tensor:
        """Cross-encoder probabilities for pre-built pair id sequences (device float32 [n])."""
        if not self._is_loaded:
            self.load()
        ids, mask = pad_batch(pairs)
        ids_t = torch.tensor(ids, dtype=torch.int32, device=self._device)
        mask_t = torch.tensor(mask, dtype=torch.int32, device=self._device)
        return self._model.forward(ids_t, mask_t)

    def score_pairs(self, query: str, texts: list[str]) -> list[float]:
        q = self.tokenizer.tokenize(query)
        pairs = [pair_ids(q, self.tokenizer.tokenize(t), self.config.max_length) for t in texts]
        return self.score_ids(pairs).cpu().tolist()

    def rerank(self, query: str, results: list[RetrievalResult],
               top_k: int | None = None) -> list[RetrievalResult]:
        if not results:
            return results
        top_k = top_k or self.config.top_k
        if len(results) <= top_k:
            return sorted(results, key=lambda x: x.score, reverse=True)
        try:
            if not self._is_loaded:
                self.load()
            scores = self.score_pairs(query, [r.chunk.text for r in results])
            reranked = [RetrievalResult(chunk=r.chunk, score=float(scores[i]))
                        for i, r in enumerate(results)]
            reranked.sort(key=lambda x: x.score, reverse=True)
            return reranked[:top_k]
        except Exception as e:
            logger.warning(f"Reranking failed: {e}, returning original top-{top_k}")
            return sorted(results, key=lambda x: x.score, reverse=True)[:top_k]
