"""A chunk collection: host staging of upserted points plus their device indexes.

Replaces one Qdrant collection as QdrantRetriever creates and fills it
(src/audio_rag/retrieval/qdrant.py:59-132 _ensure_collection, 140-225 add):
  * named dense vector "dense" (size = embedding_dim, COSINE)      -> DenseIndex (fp16 rows)
  * named sparse vector "sparse" (hybrid collections only)         -> SparseIndex (CSR)
  * payload {text, start, end, speaker, metadata}                  -> host list
Points get consecutive ordinals in upsert order (the reference's uuid4 ids are never surfaced:
RetrievalResult carries no id, core/base.py:56-61). The device indexes are rebuilt lazily on the
first search after an add; a built index is read-only, so concurrent searches are safe, and a
rebuild never frees an index a running search still holds (the old handles die with their last
reference).
"""

from __future__ import annotations

import threading
import weakref
from dataclasses import dataclass, field

import numpy as np
import torch

from audio_rag_amd.retrieval.device import DenseIndex, SparseIndex

BGE_M3_VOCAB = 250002


_NO_MATCH = object()


def _canon(x):
    """The equivalence class _match_value compares a scalar in: bools only equal bools,
    integral numbers compare by value, non-integral floats never match, strings by value.
    None when the value needs the general comparison."""
    if isinstance(x, bool):
        return ("bool", x)
    if isinstance(x, int):
        return ("num", x)
    if isinstance(x, float):
        return ("num", int(x)) if x.is_integer() else _NO_MATCH
    if isinstance(x, str):
        return ("str", x)
    return None


def _match_value(field_value, wanted) -> bool:
    """Qdrant MatchValue: equality on keyword / integer / bool payload values; an array field
    matches when any element does."""
    if isinstance(field_value, list):
        return any(_match_value(v, wanted) for v in field_value)
    if isinstance(field_value, bool) or isinstance(wanted, bool):
        return isinstance(field_value, bool) and isinstance(wanted, bool) and field_value == wanted
    if isinstance(field_value, float) and not field_value.is_integer():
        return False
    return field_value == wanted


@dataclass
class ChunkCollection:
    name: str
    dim: int
    hybrid: bool
    device: torch.device
    # host staging
    dense_rows: list[np.ndarray] = field(default_factory=list)        # fp16 [n_i, dim] blocks
    sparse_rows: list[tuple[np.ndarray, np.ndarray] | None] = field(default_factory=list)
    payloads: list[dict] = field(default_factory=list)
    # device state
    _dense: DenseIndex | None = None
    _sparse: SparseIndex | None = None
    _built_rows: int = -1
    _mask_cache: dict = field(default_factory=dict)
    _key_index: dict = field(default_factory=dict)   # metadata key -> (count, {canon: ordinals})
    _lock: threading.Lock = field(default_factory=threading.Lock)
    _frozen: bool = False
    _servers: weakref.WeakSet = field(default_factory=weakref.WeakSet)  # open StreamServers
    # captured single-query searches over the current indexes (MI355XRetriever._graph_search),
    # dropped whenever the indexes are rebuilt or closed
    _graphs: dict = field(default_factory=dict)
    # (rank, world): this process's shard of the corpus when it is spread over `world` GPUs
    # (RetrievalConfig.num_gpus): every rank stages every point on the host and builds device
    # indexes over its contiguous ordinal range only (retrieval/shards.shard_range)
    shard: tuple = (0, 1)

    def shard_bounds(self, n: int | None = None) -> tuple[int, int]:
        """[lo, hi) ordinals of this rank's shard of n (default: every) points."""
        from audio_rag_amd.retrieval.shards import shard_range

        return shard_range(self.count if n is None else n, self.shard[0], self.shard[1])

    @property
    def count(self) -> int:
        return len(self.payloads)

    # ------------------------------------------------------------------------------ upsert

    def upsert(self, dense: np.ndarray, sparse: list[tuple[np.ndarray, np.ndarray] | None],
               payloads: list[dict]) -> None:
        """dense: float16 [n, dim]; sparse[i]: (indices int32 ascending, values float32) or
        None; payloads: one dict per point."""
        if dense.dtype != np.float16 or dense.ndim != 2 or dense.shape[1] != self.dim:
            raise ValueError(f"dense vectors must be float16 [n, {self.dim}]")
        if not (len(sparse) == len(payloads) == dense.shape[0]):
            raise ValueError("dense / sparse / payload counts differ")
        if self._frozen:
            raise ValueError(f"collection {self.name} is read-only (built from device indexes)")
        bits = dense.view(np.uint16)
        if ((bits >> 10) & 31).max(initial=0) > 15:
            raise ValueError("dense components must be finite with |x| < 2 (unit embeddings)")
        with self._lock:
            self.dense_rows.append(np.ascontiguousarray(dense))
            self.sparse_rows.extend(sparse)
            self.payloads.extend(payloads)
            self._mask_cache.clear()
            self._key_index.clear()

    # ------------------------------------------------------------------------------- build

    def _ensure_built(self) -> None:
        if self._built_rows == self.count:
            return
        with self._lock:
            if self._built_rows == self.count:
                return
            rows = (np.concatenate(self.dense_rows) if self.dense_rows
                    else np.zeros((0, self.dim), dtype=np.float16))
            lo, hi = self.shard_bounds()
            old_dense, old_sparse = self._dense, self._sparse
            self._graphs = {}
            self._dense = DenseIndex(torch.from_numpy(np.ascontiguousarray(rows[lo:hi])).to(self.device),
                                     ordinal_base=lo)
            if self.hybrid:
                mine = self.sparse_rows[lo:hi]
                indptr = np.zeros(hi - lo + 1, dtype=np.int64)
                lens = [0 if s is None else len(s[0]) for s in mine]
                np.cumsum(lens, out=indptr[1:])
                idx = np.concatenate([s[0] for s in mine if s is not None] or
                                     [np.zeros(0, np.int32)]).astype(np.int32)
                val = np.concatenate([s[1] for s in mine if s is not None] or
                                     [np.zeros(0, np.float32)]).astype(np.float32)
                # the vocabulary of the whole corpus: every shard answers the same term ids
                vmax = max((int(s[0].max(initial=-1)) for s in self.sparse_rows if s is not None),
                           default=-1)
                vocab = max(BGE_M3_VOCAB, vmax + 1)
                t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.device)
                self._sparse = SparseIndex(t(indptr), t(idx), t(val), vocab, ordinal_base=lo)
            self._built_rows = self.count
            # The superseded indexes are not closed here: a search that fetched them before
            # this rebuild may still be using them. Dropping the reference frees each one (its
            # __del__ closes it) once the last such search lets go of it.
            del old_dense, old_sparse

    def query_graphs(self) -> dict:
        """The captured single-query searches of the current indexes (key -> graph)."""
        self._ensure_built()
        return self._graphs

    @property
    def dense_index(self) -> DenseIndex:
        self._ensure_built()
        return self._dense

    @property
    def sparse_index(self) -> SparseIndex | None:
        self._ensure_built()
        return self._sparse

    # ------------------------------------------------------------------------------ filter

    def filter_mask(self, filter_metadata: dict | None) -> torch.Tensor | None:
        """Bitmask (int64 words on the device) of points whose payload metadata matches every
        condition: Filter(must=[FieldCondition(key=f"metadata.{k}", match=MatchValue(v))])
        (qdrant.py:263-269). Bit r = row r of this rank's shard (ordinal lo + r)."""
        if not filter_metadata:
            return None
        key = tuple(sorted((k, repr(v)) for k, v in filter_metadata.items()))
        cached = self._mask_cache.get(key)
        if cached is not None and cached[0] == self.count:
            return cached[1]
        n = self.count
        ok = np.ones(n, dtype=bool)
        for k, v in filter_metadata.items():
            ok &= self._key_matches(k, v, n)
        lo, hi = self.shard_bounds(n)
        ok = ok[lo:hi]
        words = np.zeros(max((hi - lo + 63) // 64, 1), dtype=np.uint64)
        idx = np.nonzero(ok)[0]
        np.bitwise_or.at(words, idx >> 6, np.left_shift(np.uint64(1), (idx & 63).astype(np.uint64)))
        mask = torch.from_numpy(words.view(np.int64)).to(self.device)
        self._mask_cache[key] = (n, mask)
        return mask

    def _key_matches(self, key: str, wanted, n: int) -> np.ndarray:
        """bool [n]: points whose metadata[key] matches `wanted` (_match_value). One pass over
        the payloads per metadata key (cached until the next upsert) builds an inverted map
        value-class -> ordinals, so a new filter value costs O(matches), not O(points)."""
        cached = self._key_index.get(key)
        if cached is None or cached[0] != n:
            inv: dict = {}
            general: list[int] = []  # points whose value needs the general comparison
            for i, p in enumerate(self.payloads[:n]):
                md = p.get("metadata") or {}
                if key not in md:
                    continue
                fv = md[key]
                for x in (fv if isinstance(fv, list) else (fv,)):
                    c = _canon(x)
                    if c is None:
                        general.append(i)
                    elif c is not _NO_MATCH:
                        inv.setdefault(c, []).append(i)
            cached = (n, {c: np.unique(np.asarray(v, dtype=np.int64)) for c, v in inv.items()},
                      general)
            self._key_index[key] = cached
        _, inv, general = cached
        ok = np.zeros(n, dtype=bool)
        c = _canon(wanted)
        if c is not None and c is not _NO_MATCH and c in inv:
            ok[inv[c]] = True
        for i in general:  # rare value types (None, dicts): the reference comparison
            if not ok[i] and _match_value(self.payloads[i]["metadata"][key], wanted):
                ok[i] = True
        if c is None:  # an unusual wanted value: compare every point that has the key
            for i, p in enumerate(self.payloads[:n]):
                md = p.get("metadata") or {}
                if key in md and _match_value(md[key], wanted):
                    ok[i] = True
        return ok

    @classmethod
    def from_indexes(cls, name: str, dense: DenseIndex, payloads: list[dict],
                     sparse: SparseIndex | None = None, shard: tuple = (0, 1)) -> "ChunkCollection":
        """A read-only collection over device indexes built elsewhere (a loaded store shard, a
        synthetic benchmark corpus). Nothing is staged on the host, so it cannot be saved or
        extended with upsert(). Sharded (shard = (rank, world)): the indexes hold this rank's
        shard_range of the corpus (ordinal_base = its first ordinal), payloads every point."""
        coll = cls(name, dense.dim, sparse is not None, dense.device)
        coll.shard = tuple(shard)
        lo, hi = coll.shard_bounds(len(payloads))
        if dense.n_rows != hi - lo or dense.ordinal_base != lo:
            raise ValueError("the dense index must hold this rank's shard of the payloads "
                             f"(ordinals [{lo}, {hi}))")
        coll.payloads = payloads
        coll._dense, coll._sparse = dense, sparse
        coll._built_rows = len(payloads)
        coll._frozen = True
        return coll

    # ------------------------------------------------------------------------ persistence

    def save(self, path) -> None:
        """Writes the collection as an on-disk chunk store (retrieval/store.py)."""
        from audio_rag_amd.retrieval.store import save_arrays

        if self._frozen:
            raise ValueError(f"collection {self.name} has no host copy (built from device indexes)")
        with self._lock:
            rows = (np.concatenate(self.dense_rows) if self.dense_rows
                    else np.zeros((0, self.dim), dtype=np.float16))
            save_arrays(path, self.name, rows, list(self.sparse_rows), list(self.payloads),
                        self.hybrid)

    @classmethod
    def load(cls, path, device: torch.device, name: str | None = None) -> "ChunkCollection":
        """A collection holding every point of an on-disk chunk store, in ordinal order."""
        from audio_rag_amd.retrieval.store import load_shard

        sh = load_shard(path)
        coll = cls(name or sh.name, sh.dim, sh.hybrid, device)
        coll.upsert(np.ascontiguousarray(sh.dense, dtype=np.float16), sh.sparse_rows(),
                    sh.payloads)
        return coll

    def attach_server(self, server) -> None:
        """Registers a StreamServer over this collection's indexes: close() stops it first."""
        self._servers.add(server)

    def close(self) -> None:
        # the native servers' dispatcher threads launch searches on these indexes: stop them
        # before the indexes are freed
        for srv in list(self._servers):
            srv.close()
        self._graphs = {}
        for ix in (self._dense, self._sparse):
            if ix is not None:
                ix.close()
        self._dense = self._sparse = None
        self._built_rows = -1
