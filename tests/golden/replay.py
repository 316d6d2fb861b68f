"""Helpers shared by the golden-fixture tests (data plumbing only)."""

from __future__ import annotations

import json
from pathlib import Path

import numpy as np

import scenario

FIXTURE = Path(__file__).resolve().parent / "reference_query_path.json"
COLLECTION_HYBRID = {"ingested": True, "hybrid_real": True, "legacy": False, "empty": False}


CONFIG_FIXTURE = Path(__file__).resolve().parent / "reference_config_development.json"


def reference_config() -> dict:
    """The configuration the reference's loader builds from its own config files
    (make_config_fixture.py), as a plain dict."""
    return json.loads(CONFIG_FIXTURE.read_text())["config"]


def load():
    golden = json.loads(FIXTURE.read_text())
    s = scenario.build()
    assert golden["scenario_digest"] == scenario.digest(s), "scenario generator drifted"
    return golden, s


def sorted_sparse(lex: dict[str, float]) -> tuple[np.ndarray, np.ndarray]:
    idx = np.array([int(k) for k in lex], dtype=np.int64)
    val = np.array(list(lex.values()), dtype=np.float32)
    o = np.argsort(idx, kind="stable")
    return idx[o].astype(np.int32), val[o]


def corpus_csr(s, with_sparse: bool):
    n = len(s["chunks"])
    if not with_sparse:
        return np.zeros(n + 1, np.int64), np.zeros(0, np.int32), np.zeros(0, np.float32)
    parts = [sorted_sparse(x) for x in s["lex"]]
    indptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum([len(p[0]) for p in parts], out=indptr[1:])
    return indptr, np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts])


def query_csr(s, q: int):
    i, v = sorted_sparse(s["qlex"][q])
    return np.array([0, len(i)], dtype=np.int32), i, v


def filter_mask(s, flt: dict | None):
    if not flt:
        return None
    n = len(s["chunks"])
    words = np.zeros((n + 63) // 64, dtype=np.uint64)
    for i, c in enumerate(s["chunks"]):
        md = c["metadata"]
        if all(k in md and md[k] == v for k, v in flt.items()):
            words[i >> 6] |= np.uint64(1) << np.uint64(i & 63)
    return words


def ordinals(results) -> list[int]:
    return [r["ordinal"] for r in results]
