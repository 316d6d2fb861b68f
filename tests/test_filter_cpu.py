"""Metadata filter (qdrant.py:262-269 FieldCondition(key="metadata.<k>", MatchValue(v)), AND of
conditions): the per-key inverted index behind ChunkCollection.filter_mask selects exactly the
points the direct MatchValue comparison selects, for every value type the payloads carry."""

import random

import numpy as np
import torch

from audio_rag_amd.retrieval.collection import ChunkCollection, _match_value

VALUES = [0, 1, 2, True, False, 1.0, 2.5, "a", "b", None, [1, "a"], [True], 3.0, {"x": 1}, -1]


def _payloads(n, seed):
    rng = random.Random(seed)
    return [{"metadata": {"k": rng.choice(VALUES), "j": rng.choice(VALUES)}
             if rng.random() < 0.9 else {}} for _ in range(n)]


def test_key_index_equals_match_value():
    pay = _payloads(3000, 0)
    c = ChunkCollection("t", 4, False, torch.device("cpu"))
    c.payloads = pay
    for wanted in VALUES[:-2] + [7, "zz", 2.0, -1]:
        for key in ("k", "j", "missing"):
            got = c._key_matches(key, wanted, len(pay))
            want = np.array([key in p["metadata"] and _match_value(p["metadata"][key], wanted)
                             for p in pay])
            assert (got == want).all(), (key, wanted)


def test_filter_mask_bits_and_upsert_invalidation():
    c = ChunkCollection("t", 4, False, torch.device("cpu"))
    rows = np.zeros((130, 4), dtype=np.float16)
    c.upsert(rows, [None] * 130, [{"metadata": {"lecture": i % 3, "tag": "x" if i % 2 else "y"}}
                                  for i in range(130)])
    flt = {"lecture": 1, "tag": "x"}
    words = c.filter_mask(flt).numpy().view(np.uint64)
    bits = [(int(words[i >> 6]) >> (i & 63)) & 1 for i in range(130)]
    assert bits == [int(i % 3 == 1 and i % 2 == 1) for i in range(130)]
    c.upsert(rows[:10], [None] * 10, [{"metadata": {"lecture": 1, "tag": "x"}}] * 10)
    words = c.filter_mask(flt).numpy().view(np.uint64)
    assert sum(bin(int(w)).count("1") for w in words) == sum(bits) + 10
