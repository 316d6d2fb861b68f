"""On-disk chunk store: the persistent form of a collection, loadable whole or by shard.

Replaces the Qdrant collection the reference persists (QdrantRetriever._ensure_collection /
add, src/audio_rag/retrieval/qdrant.py:59-132, 140-225: named dense vector "dense"
VectorParams(dim, COSINE), sparse vector "sparse", payload {text, start, end, speaker,
metadata}). SURVEY.md §8(f) item 1. Layout of a store directory:

    meta.json            {"format": FORMAT, "name", "dim", "count", "hybrid", "vocab",
                          "sparse_nnz", "files": {...}}
    dense.f16            [count, dim] IEEE binary16, row-major, little-endian (the vectors exactly
                         as upserted: the canonical fp16 values the device store holds)
    sparse.indptr.i64    [count + 1]  \\
    sparse.indices.i32   [nnz]         > hybrid collections only; a point stored without a sparse
    sparse.values.f32    [nnz]        /  vector (e.g. the reference's sparse-drop) has an empty row
    payload.jsonl        one JSON object per point, ordinal order

Ordinal = row index = the order points were upserted, so a store written by one retriever and
loaded by another returns the same ordinals. Shard loading memory-maps the files and reads only
rows [lo, hi) of the dense and sparse arrays (the rank's slice of shards.shard_range); payloads
are host-replicated (every rank resolves any global ordinal).
"""

from __future__ import annotations

import json
import os
from dataclasses import dataclass
from pathlib import Path

import numpy as np

FORMAT = "armi-chunkstore-1"
FILES = {"dense": "dense.f16", "indptr": "sparse.indptr.i64", "indices": "sparse.indices.i32",
         "values": "sparse.values.f32", "payload": "payload.jsonl"}


@dataclass
class StoreShard:
    """Rows [lo, hi) of a stored collection (host arrays; memory-mapped where possible)."""

    name: str
    dim: int
    count: int             # rows of the whole store
    hybrid: bool
    vocab: int
    lo: int
    hi: int
    dense: np.ndarray      # float16 [hi - lo, dim]
    indptr: np.ndarray | None   # int64 [hi - lo + 1], rebased to 0
    indices: np.ndarray | None  # int32
    values: np.ndarray | None   # float32
    payloads: list[dict]   # all `count` payloads (host-replicated)

    def sparse_rows(self) -> list[tuple[np.ndarray, np.ndarray] | None]:
        """Per-row (indices, values), None for rows stored without a sparse vector."""
        if not self.hybrid:
            return [None] * (self.hi - self.lo)
        out = []
        for i in range(self.hi - self.lo):
            a, b = int(self.indptr[i]), int(self.indptr[i + 1])
            out.append(None if a == b else (self.indices[a:b], self.values[a:b]))
        return out


def _write_atomic(path: Path, data: bytes) -> None:
    tmp = path.with_suffix(path.suffix + ".tmp")
    with open(tmp, "wb") as f:
        f.write(data)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


def save_arrays(path: str | os.PathLike, name: str, dense: np.ndarray,
                sparse: list[tuple[np.ndarray, np.ndarray] | None] | None,
                payloads: list[dict], hybrid: bool, vocab: int = 250002) -> Path:
    """Writes a store. dense: float16 [n, dim]; sparse[i]: (ascending int32 indices, float32
    values) or None; payloads: n JSON-serialisable dicts."""
    d = Path(path)
    d.mkdir(parents=True, exist_ok=True)
    dense = np.ascontiguousarray(dense, dtype=np.float16)
    n, dim = dense.shape
    if len(payloads) != n or (sparse is not None and len(sparse) != n):
        raise ValueError("dense / sparse / payload counts differ")
    _write_atomic(d / FILES["dense"], dense.astype("<f2").tobytes())
    nnz = 0
    if hybrid:
        rows = sparse if sparse is not None else [None] * n
        lens = np.array([0 if s is None else len(s[0]) for s in rows], dtype=np.int64)
        indptr = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(lens, out=indptr[1:])
        nnz = int(indptr[-1])
        idx = np.concatenate([np.asarray(s[0], dtype=np.int32) for s in rows if s is not None]
                             or [np.zeros(0, np.int32)])
        val = np.concatenate([np.asarray(s[1], dtype=np.float32) for s in rows if s is not None]
                             or [np.zeros(0, np.float32)])
        _write_atomic(d / FILES["indptr"], indptr.astype("<i8").tobytes())
        _write_atomic(d / FILES["indices"], idx.astype("<i4").tobytes())
        _write_atomic(d / FILES["values"], val.astype("<f4").tobytes())
    lines = "".join(json.dumps(p, separators=(",", ":")) + "\n" for p in payloads)
    _write_atomic(d / FILES["payload"], lines.encode())
    meta = {"format": FORMAT, "name": name, "dim": int(dim), "count": int(n), "hybrid": bool(hybrid),
            "vocab": int(vocab), "sparse_nnz": nnz,
            "files": {k: v for k, v in FILES.items() if hybrid or k in ("dense", "payload")}}
    _write_atomic(d / "meta.json", json.dumps(meta, indent=1).encode())
    return d


def read_meta(path: str | os.PathLike) -> dict:
    meta = json.loads((Path(path) / "meta.json").read_text())
    if meta.get("format") != FORMAT:
        raise ValueError(f"{path}: not a {FORMAT} store (format={meta.get('format')!r})")
    return meta


def load_shard(path: str | os.PathLike, rank: int = 0, world: int = 1) -> StoreShard:
    """Rows of `rank` (contiguous ordinal range, shards.shard_range) of a stored collection."""
    from audio_rag_amd.retrieval.shards import shard_range

    d = Path(path)
    meta = read_meta(d)
    n, dim, hybrid = meta["count"], meta["dim"], meta["hybrid"]
    lo, hi = shard_range(n, rank, world)
    size = (d / FILES["dense"]).stat().st_size
    if size != n * dim * 2:
        raise ValueError(f"{d / FILES['dense']}: {size} bytes, expected {n * dim * 2}")
    dense = (np.memmap(d / FILES["dense"], dtype="<f2", mode="r", shape=(n, dim))[lo:hi]
             if n else np.zeros((0, dim), dtype=np.float16))
    indptr = indices = values = None
    if hybrid:
        ip = np.fromfile(d / FILES["indptr"], dtype="<i8")
        if ip.shape[0] != n + 1 or ip[-1] != meta["sparse_nnz"]:
            raise ValueError(f"{d}: sparse index pointer does not match meta.json")
        a, b = int(ip[lo]), int(ip[hi])
        nnz = meta["sparse_nnz"]
        if nnz:
            indices = np.memmap(d / FILES["indices"], dtype="<i4", mode="r", shape=(nnz,))[a:b]
            values = np.memmap(d / FILES["values"], dtype="<f4", mode="r", shape=(nnz,))[a:b]
        else:
            indices = np.zeros(0, np.int32)
            values = np.zeros(0, np.float32)
        indptr = (ip[lo:hi + 1] - a).astype(np.int64)
    with open(d / FILES["payload"], "rb") as f:
        payloads = [json.loads(line) for line in f]
    if len(payloads) != n:
        raise ValueError(f"{d}: {len(payloads)} payloads for {n} points")
    return StoreShard(meta["name"], dim, n, hybrid, meta["vocab"], lo, hi, dense, indptr, indices,
                      values, payloads)


def open_shard(path: str | os.PathLike, rank: int, world: int, device):
    """Device indexes of this rank's shard of a stored collection, for ShardedSearch:
    (DenseIndex with ordinal_base = lo, SparseIndex or None, StoreShard)."""
    import torch

    from audio_rag_amd.retrieval.device import DenseIndex, SparseIndex

    sh = load_shard(path, rank, world)
    rows = torch.from_numpy(np.ascontiguousarray(sh.dense, dtype=np.float16)).to(device)
    dense = DenseIndex(rows, ordinal_base=sh.lo)
    sparse = None
    if sh.hybrid:
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
        vocab = max(sh.vocab, int(np.max(sh.indices, initial=-1)) + 1)
        sparse = SparseIndex(t(sh.indptr.astype(np.int64)), t(sh.indices.astype(np.int32)),
                             t(sh.values.astype(np.float32)), vocab, ordinal_base=sh.lo)
    return dense, sparse, sh
