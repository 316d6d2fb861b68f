"""MI355XRetriever: drop-in replacement of QdrantRetriever (src/audio_rag/retrieval/qdrant.py).

Same constructor (config, embedding_dim), same methods and semantics:
  add(chunks, embeddings, collection_name)                      qdrant.py:140-225
  search(query_embedding, top_k, collection_name, filter_metadata, search_type)  qdrant.py:227-352
  delete_collection / count / collection_exists / is_hybrid_collection         qdrant.py:134-138, 354-381
The ranking arithmetic runs on the GPU through libarmi (dense cosine, sparse dot, RRF); nothing
falls back to the CPU. search_batch() is the batched device API the pipeline and bench use.
"""

from __future__ import annotations

import hashlib
import json
import logging
import threading
from dataclasses import dataclass

import numpy as np
import torch

from audio_rag_amd.config.schema import RetrievalConfig
from audio_rag_amd.core.base import (AudioChunk, BaseRetriever, EmbeddingResult, RetrievalResult,
                                     SparseVector)
from audio_rag_amd.core.exceptions import RetrievalError
from audio_rag_amd.retrieval.base import RetrievalRegistry
from audio_rag_amd.retrieval.collection import ChunkCollection
from audio_rag_amd.retrieval.device import ConcurrentHybrid, TopK
from audio_rag_amd.utils.decorators import timed

logger = logging.getLogger(__name__)


@dataclass
class QueryBatch:
    """B queries on the device: dense fp16 [B, dim] and an optional sparse CSR."""

    dense: torch.Tensor
    sparse_indptr: torch.Tensor | None = None   # int32 [B+1]
    sparse_indices: torch.Tensor | None = None  # int32
    sparse_values: torch.Tensor | None = None   # float32

    @property
    def has_sparse(self) -> bool:
        return self.sparse_indptr is not None


def sparse_arrays(sv: SparseVector | None) -> tuple[np.ndarray, np.ndarray] | None:
    """SparseVector -> (ascending int32 indices, float32 values). Qdrant stores sparse vectors
    sorted by index; duplicate indices are rejected like Qdrant does."""
    if sv is None:
        return None
    idx = np.asarray(sv.indices, dtype=np.int64)
    val = np.asarray(sv.values, dtype=np.float32)
    if idx.shape != val.shape:
        raise ValueError("sparse vector indices and values differ in length")
    order = np.argsort(idx, kind="stable")
    idx, val = idx[order], val[order]
    if idx.size and (np.any(idx[1:] == idx[:-1]) or idx[0] < 0 or idx[-1] >= 2**31):
        raise ValueError("sparse vector indices must be unique non-negative int32")
    return idx.astype(np.int32), val


MAX_QUERY_TERMS = 256  # armi_sparse_topk's per-query term capacity (include/armi.h)


def query_sparse_arrays(sv: SparseVector | None) -> tuple[np.ndarray, np.ndarray] | None:
    """sparse_arrays for a query vector, refusing more terms than the device search scores (it
    would silently use only the first 256; Qdrant uses every term)."""
    arr = sparse_arrays(sv)
    if arr is not None and arr[0].size > MAX_QUERY_TERMS:
        raise ValueError(f"sparse query has {arr[0].size} terms; the MI355X sparse search takes at "
                         f"most {MAX_QUERY_TERMS}")
    return arr


def fp16_rows(vectors: list[list[float]] | np.ndarray, dim: int) -> np.ndarray:
    a = np.asarray(vectors, dtype=np.float32)
    if a.ndim != 2 or a.shape[1] != dim:
        raise ValueError(f"dense vectors must have dimension {dim}, got shape {a.shape}")
    return a.astype(np.float16)


class _QueryGraph:
    """One unfiltered single-query search of a collection, captured as a HIP graph for one
    (branch, top_k): the query's dense fp16 vector and sparse terms (<= 256) are written into a
    pinned staging buffer and sent in one host->device copy, the graph replays every search
    kernel (dense scan / merge / second pass, the sparse chain on its side stream, RRF) plus the
    packing of (count, ids, scores) into one fp64 row, and one device->host copy brings that row
    back. The eager path launches the same kernels one Python call at a time, with a copy per
    input array and a packing step per result."""

    def __init__(self, ret: "MI355XRetriever", coll: ChunkCollection, mode: str, top_k: int):
        dev, dim = ret.device, coll.dim
        self.indexes = (coll.dense_index, coll.sparse_index)  # the graph's kernels read them
        self.mode, self.k, self.dim = mode, top_k, dim
        self.lock = threading.Lock()
        off_ptr = dim * 2
        off_idx = off_ptr + 16
        off_val = off_idx + 4 * MAX_QUERY_TERMS
        total = off_val + 4 * MAX_QUERY_TERMS
        self.host = torch.zeros(total, dtype=torch.uint8, pin_memory=True)
        self.stage = torch.zeros(total, dtype=torch.uint8, device=dev)
        h = self.host.numpy()
        self.h_dense = h[:off_ptr].view(np.float16)
        self.h_ptr = h[off_ptr:off_ptr + 8].view(np.int32)
        self.h_idx = h[off_idx:off_val].view(np.int32)
        self.h_val = h[off_val:].view(np.float32)
        d = self.stage
        batch = QueryBatch(dense=d[:off_ptr].view(torch.float16).view(1, dim))
        if mode in ("hybrid", "sparse"):
            batch = QueryBatch(dense=batch.dense, sparse_indptr=d[off_ptr:off_ptr + 8].view(torch.int32),
                               sparse_indices=d[off_idx:off_val].view(torch.int32),
                               sparse_values=d[off_val:].view(torch.float32))
        self.out_host = torch.zeros(1 + 2 * top_k, dtype=torch.float64, pin_memory=True)

        def run():
            out = ret._search_device(coll, batch, top_k, mode, None)
            sc = out.rank if mode == "hybrid" else out.scores
            return torch.cat([out.count[:1].double(), out.ids[0].double(), sc[0].double()])

        # captured under inference mode, as the reranker's graphs are (xlmr.py forward): the
        # CUDA generator's graph-state tensors are created by the first capture in a process and
        # updated in place by every later one, which torch refuses across the two modes. The
        # warm-up query is a one-hot vector with no sparse terms: the all-zero staging buffer
        # ties every row at cosine 0, whose top-k cannot be certified, and each warm-up call then
        # ran the collect pass over the whole shard (~0.16 s at 1M rows)
        batch.dense[0, 0] = 1.0
        with torch.inference_mode():
            side = torch.cuda.Stream(device=dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(2):
                    run()
            torch.cuda.current_stream(dev).wait_stream(side)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.packed = run()

    def search(self, dense, sparse: tuple[np.ndarray, np.ndarray] | None) -> np.ndarray:
        """The packed result row (count, ids[k], scores[k]) of one query."""
        with self.lock:
            self.h_dense[:] = dense
            if sparse is not None:
                n = sparse[0].size
                self.h_ptr[0], self.h_ptr[1] = 0, n
                self.h_idx[:n] = sparse[0]
                self.h_val[:n] = sparse[1]
            stream = torch.cuda.current_stream(self.stage.device)
            self.stage.copy_(self.host, non_blocking=True)
            self.graph.replay()
            self.out_host.copy_(self.packed, non_blocking=True)
            stream.synchronize()
            return self.out_host.numpy().copy()


@RetrievalRegistry.register("mi355x")
class MI355XRetriever(BaseRetriever):
    """Dense (cosine), sparse (lexical) and hybrid (RRF) search on an MI355X chunk store."""

    def __init__(self, config: RetrievalConfig, embedding_dim: int = 1024):
        self.config = config
        self.embedding_dim = embedding_dim
        self.device = torch.device("cuda", config.device)
        self._collections: dict[str, ChunkCollection] = {}
        self._hybrid: ConcurrentHybrid | None = None
        self._graphs_ok = True  # cleared when a capture is refused (search() then runs eagerly)
        self.last_sharded = None  # the ShardedSearch of the last collective call (diagnostics)
        # num_gpus > 1: the corpus is sharded by ordinal over the ranks of the default process
        # group (one process per GPU, launched by torchrun, torch.distributed initialised and
        # the process's GPU selected before the retriever is built): see _search_sharded
        self._rank, self._world = 0, 1
        if config.num_gpus > 1:
            import torch.distributed as dist

            if not dist.is_available() or not dist.is_initialized():
                raise RetrievalError("num_gpus > 1 needs torch.distributed initialised (one "
                                     "process per GPU, e.g. torchrun) before the retriever")
            if dist.get_world_size() != config.num_gpus:
                raise RetrievalError(f"num_gpus = {config.num_gpus} but the process group has "
                                     f"{dist.get_world_size()} ranks")
            self._rank, self._world = dist.get_rank(), dist.get_world_size()
            self.device = torch.device("cuda", torch.cuda.current_device())
        logger.info(f"MI355XRetriever initialized: collection={config.collection_name}, "
                    f"search_type={config.search_type}, device={self.device}")

    # ---------------------------------------------------------------------- collections

    def _resolve_collection(self, collection_name: str | None) -> str:
        return collection_name or self.config.collection_name

    def _ensure_collection(self, collection_name: str | None = None, hybrid: bool = False) -> str:
        """Creates a missing collection (hybrid = dense + sparse named vectors, else dense-only
        legacy schema), as qdrant.py:59-132 does."""
        resolved = self._resolve_collection(collection_name)
        coll = self._collections.get(resolved)
        if coll is not None:
            if hybrid and not coll.hybrid:
                logger.warning(f"Collection {resolved} exists but is not hybrid-enabled. "
                               "Re-index required for hybrid search.")
            return resolved
        try:
            coll = ChunkCollection(resolved, self.embedding_dim, hybrid, self.device)
            coll.shard = (self._rank, self._world)
            self._collections[resolved] = coll
            logger.info(f"Creating {'hybrid' if hybrid else 'dense'} collection: {resolved}")
            return resolved
        except Exception as e:
            raise RetrievalError(f"Failed to ensure collection '{resolved}': {e}")

    def is_hybrid_collection(self, collection_name: str | None = None) -> bool:
        resolved = self._ensure_collection(collection_name)
        return self._collections[resolved].hybrid

    def delete_collection(self, collection_name: str | None = None) -> None:
        resolved = self._resolve_collection(collection_name)
        try:
            coll = self._collections.pop(resolved, None)
            if coll is not None:
                coll.close()
            logger.info(f"Deleted collection: {resolved}")
        except Exception as e:
            raise RetrievalError(f"Failed to delete collection '{resolved}': {e}")

    def count(self, collection_name: str | None = None) -> int:
        resolved = self._ensure_collection(collection_name)
        return self._collections[resolved].count

    def collection_exists(self, collection_name: str | None = None) -> bool:
        return self._resolve_collection(collection_name) in self._collections

    def collection(self, collection_name: str | None = None) -> ChunkCollection:
        return self._collections[self._ensure_collection(collection_name)]

    # ------------------------------------------------------------------------------ add

    @timed
    def add(self, chunks: list[AudioChunk], embeddings: list[EmbeddingResult],
            collection_name: str | None = None) -> None:
        if not chunks:
            return
        if len(chunks) != len(embeddings):
            raise RetrievalError(f"Chunks/embeddings mismatch: {len(chunks)} chunks, "
                                 f"{len(embeddings)} embeddings")
        has_sparse = any(e.sparse is not None for e in embeddings)
        resolved = self._ensure_collection(collection_name, hybrid=has_sparse)
        try:
            coll = self._collections[resolved]
            dense = fp16_rows([e.dense for e in embeddings], self.embedding_dim)
            if coll.hybrid and not self.config.reproduce_sparse_drop:
                sparse = [sparse_arrays(e.sparse) for e in embeddings]
            else:
                # legacy collections keep dense only; with reproduce_sparse_drop the reference's
                # final dense-only batch upsert (qdrant.py:210-220) replaces every point, so the
                # stored points have no sparse vector
                sparse = [None] * len(embeddings)
            payloads = [{"text": c.text, "start": c.start, "end": c.end, "speaker": c.speaker,
                         "metadata": c.metadata or {}} for c in chunks]
            coll.upsert(dense, sparse, payloads)
            logger.info(f"Added {len(chunks)} chunks to {resolved} (hybrid={coll.hybrid})")
        except Exception as e:
            raise RetrievalError(f"Failed to add chunks to '{resolved}': {e}")

    def add_arrays(self, dense: np.ndarray, payloads: list[dict],
                   sparse: list[tuple[np.ndarray, np.ndarray] | None] | None = None,
                   collection_name: str | None = None) -> None:
        """Bulk upsert of pre-embedded chunks (fp16 [n, dim] + payload dicts), the fast ingest
        path for large corpora."""
        resolved = self._ensure_collection(collection_name, hybrid=sparse is not None)
        coll = self._collections[resolved]
        if sparse is None or not coll.hybrid:
            sparse = [None] * len(payloads)
        coll.upsert(np.ascontiguousarray(dense, dtype=np.float16), sparse, payloads)

    # ---------------------------------------------------------------------- persistence

    def save_collection(self, path, collection_name: str | None = None) -> None:
        """Persists a collection as an on-disk chunk store (retrieval/store.py), the durable
        form of the Qdrant collection qdrant.py:59-225 maintains."""
        resolved = self._resolve_collection(collection_name)
        if resolved not in self._collections:
            raise RetrievalError(f"Collection '{resolved}' does not exist")
        try:
            self._collections[resolved].save(path)
        except Exception as e:
            raise RetrievalError(f"Failed to save collection '{resolved}': {e}")

    def attach_collection(self, coll: ChunkCollection) -> None:
        """Registers a collection built elsewhere (ChunkCollection.from_indexes)."""
        old = self._collections.pop(coll.name, None)
        if old is not None and old is not coll:
            old.close()
        self._collections[coll.name] = coll

    def load_collection(self, path, collection_name: str | None = None) -> str:
        """Loads an on-disk chunk store as a collection (replacing one of the same name);
        returns the collection name."""
        try:
            from audio_rag_amd.retrieval.store import read_meta

            resolved = collection_name or read_meta(path)["name"]
            coll = ChunkCollection.load(path, self.device, resolved)
            coll.shard = (self._rank, self._world)
        except Exception as e:
            raise RetrievalError(f"Failed to load chunk store '{path}': {e}")
        old = self._collections.pop(resolved, None)
        if old is not None:
            old.close()
        self._collections[resolved] = coll
        logger.info(f"Loaded collection {resolved}: {coll.count} points (hybrid={coll.hybrid})")
        return resolved

    # --------------------------------------------------------------------------- search

    def _mode(self, coll: ChunkCollection, search_type: str, has_sparse: bool) -> str:
        if search_type == "hybrid" and coll.hybrid and has_sparse:
            return "hybrid"
        if search_type == "sparse" and coll.hybrid and has_sparse:
            return "sparse"
        return "dense" if coll.hybrid else "legacy_dense"

    def search_batch(self, queries: QueryBatch, top_k: int | None = None,
                     collection_name: str | None = None, filter_metadata: dict | None = None,
                     search_type: str | None = None) -> tuple[TopK, str]:
        """Device top-k for B queries; returns (TopK, mode). Scores are cosine (dense),
        sparse dot (sparse) or the RRF score (hybrid), as Qdrant's hit.score."""
        resolved = self._ensure_collection(collection_name)
        top_k = top_k or self.config.top_k
        search_type = search_type or self.config.search_type
        coll = self._collections[resolved]
        mode = self._mode(coll, search_type, queries.has_sparse)
        mask = coll.filter_mask(filter_metadata)
        if self._world > 1:
            return self._search_sharded(coll, queries, top_k, mode, mask, filter_metadata), mode
        return self._search_device(coll, queries, top_k, mode, mask), mode

    def _search_sharded(self, coll: ChunkCollection, queries: QueryBatch, top_k: int, mode: str,
                        mask: torch.Tensor | None, mask_spec: dict | None = None) -> TopK:
        """search_batch over the corpus sharded across the process group (num_gpus > 1), a
        COLLECTIVE call: every rank calls it with its own queries (any batch size, any branch)
        and the same top_k, collection and filter, and gets the global top-k of its own queries.
        retrieval/shards.ShardedSearch: one RCCL all-gather of all ranks' queries, the local
        kernels over this rank's shard for all of them, one all-gather of the per-shard lists,
        the merge of this rank's queries (armi_topk_merge_shards_packed), RRF after the merge
        for hybrid. Keys are exact and tie-broken by the global ordinal, so the answer equals
        the single-GPU one. Reranking stays local: each rank reranks its own queries' candidates
        (the query slice), with no further exchange."""
        from audio_rag_amd.retrieval.device import merge_shards, merge_shards_packed, rrf_fuse
        from audio_rag_amd.retrieval.shards import ShardedSearch

        sh = ShardedSearch(lambda q, k: coll.dense_index.topk(q, k, row_mask=mask), merge_shards,
                           local_sparse=(lambda c, k: coll.sparse_index.topk(*c, k, row_mask=mask))
                           if coll.hybrid else None,
                           rrf=lambda a, b, k: rrf_fuse(a, b, k, rrf_k=self.config.rrf_k),
                           merge_packed=merge_shards_packed)
        self.last_sharded = sh
        csr = (queries.sparse_indptr, queries.sparse_indices, queries.sparse_values)
        # the ranks agree on top_k and on collection + filter through the call's header (a
        # mismatch raises on every rank); batch sizes and branches may differ
        key = json.dumps([coll.name, coll.count, coll.hybrid, mask_spec or {}],
                         sort_keys=True, default=str)
        digest = int.from_bytes(hashlib.sha256(key.encode()).digest()[:8], "little")
        try:
            return sh.search(queries.dense, csr if queries.has_sparse else None, mode, top_k,
                             digest)
        except ValueError as e:
            raise RetrievalError(str(e))

    def _search_device(self, coll: ChunkCollection, queries: QueryBatch, top_k: int, mode: str,
                       mask: torch.Tensor | None) -> TopK:
        """The device work of search_batch for a resolved collection and branch."""
        if mode == "hybrid":
            if self._hybrid is None:
                self._hybrid = ConcurrentHybrid(self.device)
            sq = (queries.sparse_indptr, queries.sparse_indices, queries.sparse_values)
            fused = self._hybrid(
                lambda: coll.dense_index.topk(queries.dense, 2 * top_k, row_mask=mask),
                lambda: coll.sparse_index.topk(*sq, 2 * top_k, row_mask=mask),
                sq + ((mask,) if mask is not None else ()), top_k, rrf_k=self.config.rrf_k)
            return fused
        if mode == "sparse":
            return coll.sparse_index.topk(queries.sparse_indptr, queries.sparse_indices,
                                          queries.sparse_values, top_k, row_mask=mask)
        return coll.dense_index.topk(queries.dense, top_k, row_mask=mask)

    def to_query_batch(self, query_embeddings: list[EmbeddingResult]) -> QueryBatch:
        dense = torch.from_numpy(fp16_rows([q.dense for q in query_embeddings],
                                           self.embedding_dim)).to(self.device)
        if any(q.sparse is None for q in query_embeddings):
            return QueryBatch(dense=dense)
        parts = [query_sparse_arrays(q.sparse) for q in query_embeddings]
        indptr = np.zeros(len(parts) + 1, dtype=np.int32)
        np.cumsum([len(p[0]) for p in parts], out=indptr[1:])
        # one unused entry past indptr[-1] keeps the term arrays' device pointers non-null when
        # every query is an empty SparseVector (the C ABI refuses null arrays)
        idx = np.concatenate([p[0] for p in parts] + [np.zeros(1, np.int32)]).astype(np.int32)
        val = np.concatenate([p[1] for p in parts] + [np.zeros(1, np.float32)]).astype(np.float32)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.device)
        return QueryBatch(dense=dense, sparse_indptr=t(indptr), sparse_indices=t(idx),
                          sparse_values=t(val))

    def materialize(self, out: TopK, mode: str, resolved: str, b: int = 0,
                    threshold: float | None = None) -> list[RetrievalResult]:
        """Row b of a device TopK -> fresh RetrievalResult objects from the payload table
        (qdrant.py:334-346)."""
        coll = self._collections[resolved]
        # one packed device-to-host copy (count, ids, scores as fp64: ordinals < 2^31 and fp32
        # scores convert exactly) instead of three synchronising copies
        sc = out.rank if mode == "hybrid" else out.scores
        packed = torch.cat([out.count[b:b + 1].double(), out.ids[b].double(),
                            sc[b].double()]).cpu().numpy()
        k = out.ids.shape[1]
        count = int(packed[0])
        ids = packed[1:1 + count].astype(np.int64).tolist()
        scores = packed[1 + k:1 + k + count].tolist()
        results = []
        for pid, score in zip(ids, scores):
            if threshold is not None and score < threshold:
                continue
            p = coll.payloads[pid]
            chunk = AudioChunk(text=p.get("text", ""), start=p.get("start", 0.0),
                               end=p.get("end", 0.0), speaker=p.get("speaker"),
                               metadata=p.get("metadata"))
            results.append(RetrievalResult(chunk=chunk, score=float(score), source=resolved))
        return results

    def materialize_batch(self, out: TopK, mode: str, resolved: str,
                          threshold: float | None = None) -> list[list[RetrievalResult]]:
        """Every row of a device TopK -> RetrievalResult lists, with one device-to-host copy per
        tensor for the whole batch (materialize() copies per row)."""
        coll = self._collections[resolved]
        counts = out.count.cpu().tolist()
        ids = out.ids.cpu().tolist()
        scores = (out.rank if mode == "hybrid" else out.scores).cpu().tolist()
        batch = []
        for c, row_ids, row_sc in zip(counts, ids, scores):
            results = []
            for pid, score in zip(row_ids[:c], row_sc[:c]):
                if threshold is not None and score < threshold:
                    continue
                p = coll.payloads[pid]
                chunk = AudioChunk(text=p.get("text", ""), start=p.get("start", 0.0),
                                   end=p.get("end", 0.0), speaker=p.get("speaker"),
                                   metadata=p.get("metadata"))
                results.append(RetrievalResult(chunk=chunk, score=float(score), source=resolved))
            batch.append(results)
        return batch

    def _graph_search(self, coll: ChunkCollection, query: EmbeddingResult, top_k: int,
                      search_type: str) -> tuple[np.ndarray, str] | None:
        """search() of one unfiltered query through the collection's captured graph for its
        branch (captured on first use); None when the path does not apply."""
        if not (self.config.query_graphs and self._graphs_ok) or coll.count == 0 or self._world > 1:
            return None
        mode = self._mode(coll, search_type, query.sparse is not None)
        sparse = query_sparse_arrays(query.sparse) if mode in ("hybrid", "sparse") else None
        dense = np.asarray(query.dense, dtype=np.float32)
        if dense.shape != (self.embedding_dim,):
            raise ValueError(f"dense vectors must have dimension {self.embedding_dim}, "
                             f"got shape {(1,) + dense.shape}")
        graphs = coll.query_graphs()
        key = (mode, top_k, self.config.rrf_k)
        g = graphs.get(key)
        if g is None:
            try:
                g = _QueryGraph(self, coll, mode, top_k)
            except RuntimeError as e:  # capture refused: the same kernels through search_batch
                logger.warning(f"query graph capture failed ({e}); searching without graphs")
                self._graphs_ok = False
                return None
            graphs[key] = g
        return g.search(dense, sparse), mode

    def _materialize_packed(self, packed: np.ndarray, resolved: str, k: int,
                            threshold: float | None) -> list[RetrievalResult]:
        coll = self._collections[resolved]
        count = int(packed[0])
        ids = packed[1:1 + count].astype(np.int64).tolist()
        scores = packed[1 + k:1 + k + count].tolist()
        results = []
        for pid, score in zip(ids, scores):
            if threshold is not None and score < threshold:
                continue
            p = coll.payloads[pid]
            chunk = AudioChunk(text=p.get("text", ""), start=p.get("start", 0.0),
                               end=p.get("end", 0.0), speaker=p.get("speaker"),
                               metadata=p.get("metadata"))
            results.append(RetrievalResult(chunk=chunk, score=float(score), source=resolved))
        return results

    @timed
    def search(self, query_embedding: EmbeddingResult, top_k: int | None = None,
               collection_name: str | None = None, filter_metadata: dict | None = None,
               search_type: str | None = None) -> list[RetrievalResult]:
        resolved = self._ensure_collection(collection_name)
        top_k = top_k or self.config.top_k
        search_type = search_type or self.config.search_type
        try:
            if not filter_metadata:
                coll = self._collections[resolved]
                got = self._graph_search(coll, query_embedding, top_k, search_type)
                if got is not None:
                    packed, mode = got
                    thr = None
                    if mode == "legacy_dense" and self.config.score_threshold > 0:
                        thr = self.config.score_threshold
                    results = self._materialize_packed(packed, resolved, top_k, thr)
                    logger.debug(f"Search returned {len(results)} results")
                    return results
            batch = self.to_query_batch([query_embedding])
            out, mode = self.search_batch(batch, top_k, resolved, filter_metadata, search_type)
            thr = None
            if mode == "legacy_dense" and self.config.score_threshold > 0:
                thr = self.config.score_threshold
            results = self.materialize(out, mode, resolved, 0, thr)
            logger.debug(f"Search returned {len(results)} results")
            return results
        except Exception as e:
            raise RetrievalError(f"Search failed in '{resolved}': {e}")


# The reference's own configs name the backend "qdrant" (configs/base.yaml:39,
# config/schema.py:60); in this package that key builds the MI355X chunk store, so a reference
# deployment's YAML runs unchanged (the qdrant_host / qdrant_port / qdrant_in_memory knobs are
# accepted and ignored).
RetrievalRegistry.register("qdrant")(MI355XRetriever)
