"""BGEReranker on the MI355X (mirrors src/audio_rag/reranking/bge.py:14-147).

rerank() keeps the reference's rules exactly:
  * empty input -> returned as is; len(results) <= top_k -> sorted by retrieval score, no model
    (bge.py:104-109)
  * otherwise score every (query, chunk.text) pair with the cross-encoder (sigmoid of the
    logit), build fresh RetrievalResult(chunk, score) with source=None (bge.py:116-131),
    stable sort descending, keep top_k (bge.py:134, 141)
  * any failure -> warning + the retrieval results sorted by score, top_k (bge.py:143-147)
Weights: BAAI/bge-reranker-base is not on disk; the model is initialised from
RerankingConfig.seed. Token ids: audio_rag_amd.text (stand-in tokenizer) or rerank_ids().
"""

from __future__ import annotations

import logging

import torch

from audio_rag_amd.config.schema import RerankingConfig
from audio_rag_amd.core.base import RetrievalResult
from audio_rag_amd.core.exceptions import RerankingError
from audio_rag_amd.reranking.base import BaseReranker, RerankerRegistry
from audio_rag_amd.reranking.xlmr import CrossEncoderXLMR, build_reranker
from audio_rag_amd.text import HashTokenizer, pad_batch, pair_ids

logger = logging.getLogger(__name__)


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
        self.tokenizer = HashTokenizer()

    @property
    def vram_required(self) -> float:
        return self.MODEL_VRAM.get(self.config.model, 1.0)

    def load(self) -> None:
        if self._is_loaded:
            return
        try:
            hf = build_reranker(self.config.seed, self._arch)
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
