"""Token ids for the XLM-RoBERTa encoders of the query path.

The reference tokenises with the BAAI/bge-m3 / BAAI/bge-reranker-base sentencepiece models
(inside FlagEmbedding and sentence-transformers: embeddings/bge.py:141-147,
reranking/bge.py:119-123). Those files are not on disk and cannot be fetched, so this module is
a deterministic STAND-IN with the same vocabulary size and special ids (<s>=0, <pad>=1, </s>=2,
<unk>=3, 250002 ids): words and punctuation are hashed into [4, vocab). It reproduces the
sequence layout the reference feeds its models, not sentencepiece's segmentation:
  query encode  <s> q </s>                 (BGE-M3, max_length 8192)
  rerank pair   <s> q </s></s> d </s>      (CrossEncoder, truncation="longest_first", 512)
Every model entry point also accepts token ids directly, which is how parity is tested.
"""

from __future__ import annotations

import re

import xxhash

BOS, PAD, EOS, UNK = 0, 1, 2, 3
SPECIAL_IDS = frozenset((BOS, PAD, EOS, UNK))
VOCAB = 250002
_WORD = re.compile(r"\w+|[^\w\s]", re.UNICODE)


class HashTokenizer:
    special_ids = SPECIAL_IDS

    def __init__(self, vocab_size: int = VOCAB):
        self.vocab_size = vocab_size

    def tokenize(self, text: str) -> list[int]:
        out = []
        for w in _WORD.findall(text.lower()):
            out.append(4 + xxhash.xxh64_intdigest(w.encode("utf-8")) % (self.vocab_size - 4))
        return out

    def encode(self, text: str, max_length: int = 8192) -> list[int]:
        ids = self.tokenize(text)[: max(max_length - 2, 0)]
        return [BOS, *ids, EOS]

    def encode_pair(self, a: str | list[int], b: str | list[int], max_length: int = 512) -> list[int]:
        ta = self.tokenize(a) if isinstance(a, str) else list(a)
        tb = self.tokenize(b) if isinstance(b, str) else list(b)
        return pair_ids(ta, tb, max_length)


def pair_ids(ta: list[int], tb: list[int], max_length: int = 512) -> list[int]:
    """<s> a </s></s> b </s>, truncating token by token from the longer side (HF
    truncation="longest_first") so that the total fits max_length."""
    budget = max_length - 4
    ta, tb = list(ta), list(tb)
    while len(ta) + len(tb) > budget:
        if len(ta) > len(tb):
            ta.pop()
        else:
            tb.pop()
    return [BOS, *ta, EOS, EOS, *tb, EOS]


def pad_batch(seqs: list[list[int]], pad_to: int | None = None) -> tuple[list[list[int]], list[list[int]]]:
    """Right-pads with <pad>; returns (ids, attention mask)."""
    L = max([len(s) for s in seqs] + [pad_to or 0])
    ids = [s + [PAD] * (L - len(s)) for s in seqs]
    mask = [[1] * len(s) + [0] * (L - len(s)) for s in seqs]
    return ids, mask
