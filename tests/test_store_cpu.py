"""On-disk chunk store (audio_rag_amd/retrieval/store.py) on the CPU: exact round trips of the
vectors, sparse rows and payloads a collection was given, shard slicing, format checks, and
the retriever's save/load surface including the reference's sparse-drop switch
(QdrantRetriever.add, src/audio_rag/retrieval/qdrant.py:183-220). No device work."""

import json

import numpy as np
import pytest
import torch


def _points(n, dim=64, seed=0, none_every=3):
    rng = np.random.default_rng(seed)
    dense = rng.standard_normal((n, dim)).astype(np.float32)
    dense /= np.linalg.norm(dense, axis=1, keepdims=True)
    dense = dense.astype(np.float16)
    sparse = []
    for i in range(n):
        if none_every and i % none_every == 2:
            sparse.append(None)  # a point stored without a sparse vector
            continue
        k = int(rng.integers(1, 20))
        idx = np.sort(rng.choice(250000, size=k, replace=False)).astype(np.int32) + 4
        sparse.append((idx, rng.uniform(0.01, 0.4, size=k).astype(np.float32)))
    payloads = [{"text": f"chunk {i}", "start": float(i), "end": i + 0.5,
                 "speaker": None if i % 2 else "SPEAKER_00",
                 "metadata": {"lecture": i % 4, "tags": ["a", "b"][: i % 3]}} for i in range(n)]
    return dense, sparse, payloads


def _collection(n, hybrid=True):
    from audio_rag_amd.retrieval.collection import ChunkCollection

    dense, sparse, payloads = _points(n)
    c = ChunkCollection("lectures", dense.shape[1], hybrid, torch.device("cpu"))
    half = n // 2  # two upserts: ordinals continue across calls
    c.upsert(dense[:half], sparse[:half] if hybrid else [None] * half, payloads[:half])
    c.upsert(dense[half:], sparse[half:] if hybrid else [None] * (n - half), payloads[half:])
    return c, dense, sparse, payloads


def _same_sparse(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        if x is None or y is None:
            assert x is None and y is None
        else:
            np.testing.assert_array_equal(np.asarray(x[0]), np.asarray(y[0]))
            np.testing.assert_array_equal(np.asarray(x[1]), np.asarray(y[1]))


@pytest.mark.parametrize("hybrid", [True, False])
def test_collection_round_trip(tmp_path, hybrid):
    from audio_rag_amd.retrieval.collection import ChunkCollection
    from audio_rag_amd.retrieval.store import read_meta

    c, dense, sparse, payloads = _collection(37, hybrid)
    c.save(tmp_path / "s")
    meta = read_meta(tmp_path / "s")
    assert meta["count"] == 37 and meta["dim"] == 64 and meta["hybrid"] == hybrid
    d = ChunkCollection.load(tmp_path / "s", torch.device("cpu"))
    assert d.name == "lectures" and d.count == 37 and d.hybrid == hybrid
    got = np.concatenate(d.dense_rows)
    assert got.dtype == np.float16
    np.testing.assert_array_equal(got.view(np.uint16), dense.view(np.uint16))  # bit-exact
    assert d.payloads == payloads
    _same_sparse(d.sparse_rows, sparse if hybrid else [None] * 37)


def test_shards_tile_the_store(tmp_path):
    from audio_rag_amd.retrieval.store import load_shard

    c, dense, sparse, payloads = _collection(50)
    c.save(tmp_path / "s")
    world = 3
    rows, rebuilt = [], []
    for r in range(world):
        sh = load_shard(tmp_path / "s", r, world)
        assert sh.count == 50 and len(sh.payloads) == 50  # payloads host-replicated
        assert sh.indptr[0] == 0 and sh.indptr[-1] == len(sh.indices)
        rows.append(np.asarray(sh.dense))
        rebuilt += sh.sparse_rows()
        assert (sh.lo, sh.hi) == (50 * r // world, 50 * (r + 1) // world)
    np.testing.assert_array_equal(np.concatenate(rows).view(np.uint16), dense.view(np.uint16))
    _same_sparse(rebuilt, sparse)


def test_format_checks(tmp_path):
    from audio_rag_amd.retrieval.store import load_shard, save_arrays

    dense, sparse, payloads = _points(5)
    with pytest.raises(ValueError, match="counts differ"):
        save_arrays(tmp_path / "bad", "x", dense, sparse, payloads[:4], True)
    save_arrays(tmp_path / "s", "x", dense, sparse, payloads, True)
    meta = json.loads((tmp_path / "s" / "meta.json").read_text())
    meta["format"] = "something-else"
    (tmp_path / "s" / "meta.json").write_text(json.dumps(meta))
    with pytest.raises(ValueError, match="not a"):
        load_shard(tmp_path / "s")
    save_arrays(tmp_path / "t", "x", dense, sparse, payloads, True)
    with open(tmp_path / "t" / "dense.f16", "ab") as f:
        f.write(b"\0\0")
    with pytest.raises(ValueError, match="bytes, expected"):
        load_shard(tmp_path / "t")
    empty = save_arrays(tmp_path / "e", "x", np.zeros((0, 8), np.float16), [], [], True)
    sh = load_shard(empty)
    assert sh.count == 0 and sh.dense.shape == (0, 8) and sh.sparse_rows() == []


@pytest.mark.parametrize("drop", [False, True])
def test_retriever_save_load_and_sparse_drop(tmp_path, drop):
    """add() -> save_collection -> load_collection in a fresh retriever keeps every point; with
    reproduce_sparse_drop the stored points have no sparse vector, as Qdrant holds them after
    the reference's dense-only re-upsert."""
    from audio_rag_amd.config import RetrievalConfig
    from audio_rag_amd.core import AudioChunk, EmbeddingResult, SparseVector
    from audio_rag_amd.retrieval.mi355x import MI355XRetriever

    dense, sparse, payloads = _points(12, dim=1024, none_every=0)
    chunks = [AudioChunk(text=p["text"], start=p["start"], end=p["end"], speaker=p["speaker"],
                         metadata=p["metadata"]) for p in payloads]
    embs = [EmbeddingResult(dense=dense[i].astype(np.float32).tolist(),
                            sparse=SparseVector(sparse[i][0].tolist(), sparse[i][1].tolist()))
            for i in range(12)]
    cfg = RetrievalConfig(reproduce_sparse_drop=drop)
    a = MI355XRetriever(cfg, embedding_dim=1024)
    a.add(chunks, embs, collection_name="c1")
    a.save_collection(tmp_path / "c1", collection_name="c1")
    b = MI355XRetriever(cfg, embedding_dim=1024)
    assert b.load_collection(tmp_path / "c1") == "c1"
    assert b.count("c1") == 12 and b.is_hybrid_collection("c1")
    coll = b.collection("c1")
    np.testing.assert_array_equal(np.concatenate(coll.dense_rows).view(np.uint16),
                                  dense.view(np.uint16))
    if drop:
        assert all(s is None for s in coll.sparse_rows)
    else:
        _same_sparse(coll.sparse_rows, sparse)
    assert coll.payloads[3]["metadata"] == {"lecture": 3, "tags": []}


def test_query_sparse_vectors_are_sorted_and_capped():
    """Query CSRs reach armi_sparse_topk ascending and unique; a query with more terms than the
    device search scores (256) is refused instead of silently truncated."""
    from audio_rag_amd.core import SparseVector
    from audio_rag_amd.retrieval.mi355x import MAX_QUERY_TERMS, query_sparse_arrays

    idx, val = query_sparse_arrays(SparseVector(indices=[9, 4, 7], values=[0.1, 0.2, 0.3]))
    assert idx.tolist() == [4, 7, 9] and val.tolist() == pytest.approx([0.2, 0.3, 0.1])
    assert query_sparse_arrays(None) is None
    ok = SparseVector(indices=list(range(4, 4 + MAX_QUERY_TERMS)), values=[0.1] * MAX_QUERY_TERMS)
    assert query_sparse_arrays(ok)[0].size == MAX_QUERY_TERMS
    long = SparseVector(indices=list(range(4, 5 + MAX_QUERY_TERMS)), values=[0.1] * (MAX_QUERY_TERMS + 1))
    with pytest.raises(ValueError, match="at most 256"):
        query_sparse_arrays(long)
    with pytest.raises(ValueError, match="unique"):
        query_sparse_arrays(SparseVector(indices=[5, 5], values=[0.1, 0.2]))
