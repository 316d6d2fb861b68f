"""QueryBatcher (audio_rag_amd/retrieval/batcher.py) on the CPU with a recording stand-in for
MI355XRetriever.search_batch: every concurrent caller gets its own query's answer, batches
respect max_batch, requests with different filters or sparse/dense-only never share a batch,
and a failing search fails every caller of its batch with RetrievalError (as search() raises).
The device search itself is covered by tests/test_batcher_gpu.py."""

import threading

import numpy as np
import pytest
import torch

from audio_rag_amd.config import RetrievalConfig
from audio_rag_amd.core import AudioChunk, RetrievalResult
from audio_rag_amd.core.exceptions import RetrievalError
from audio_rag_amd.retrieval.device import TopK


class FakeRetriever:
    """search_batch answers query b with the single id round(dense[b, 0] * 1000)."""

    def __init__(self, fail=False):
        self.device = torch.device("cpu")
        self.config = RetrievalConfig()
        self.calls = []
        self.fail = fail
        self.lock = threading.Lock()

    def _resolve_collection(self, name):
        return name or "audio_rag"

    def search_batch(self, qb, top_k, resolved, filt, search_type):
        with self.lock:
            self.calls.append((qb.dense.shape[0], filt, qb.has_sparse))
        if self.fail:
            raise RuntimeError("device lost")
        ids = torch.round(qb.dense[:, :1].float() * 1000).to(torch.int64)
        n = ids.shape[0]
        return TopK(scores=torch.ones(n, 1), ids=ids, rank=torch.ones(n, 1, dtype=torch.float64),
                    count=torch.ones(n, dtype=torch.int32)), "dense"

    def materialize_batch(self, out, mode, resolved, threshold=None):
        return [[RetrievalResult(AudioChunk(text=str(int(i)), start=0, end=0), 1.0, resolved)]
                for i in out.ids[:, 0].tolist()]


def _vec(i, dim=16):
    v = np.zeros(dim, dtype=np.float32)
    v[0] = i / 1000.0
    return v


def test_concurrent_callers_get_their_own_answers():
    from audio_rag_amd.retrieval.batcher import QueryBatcher

    fr = FakeRetriever()
    futs = {}
    with QueryBatcher(fr, max_batch=8, max_wait_ms=5.0) as qb:
        def client(base):
            for i in range(base, base + 50):
                futs[i] = qb.submit_arrays(_vec(i))
        ts = [threading.Thread(target=client, args=(b,)) for b in (0, 100, 200, 300)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        for i, f in futs.items():
            assert f.result(timeout=10)[0].chunk.text == str(i)
    assert sum(c[0] for c in fr.calls) == 200
    assert all(c[0] <= 8 for c in fr.calls)
    assert len(fr.calls) < 200  # actually batched


def test_groups_never_mix_filters_or_sparse():
    from audio_rag_amd.retrieval.batcher import QueryBatcher

    fr = FakeRetriever()
    qb = QueryBatcher(fr, max_batch=64, max_wait_ms=50.0)
    fs = [qb.submit_arrays(_vec(1), None, {"lecture": 1}),
          qb.submit_arrays(_vec(2), None, None),
          qb.submit_arrays(_vec(3), (np.array([5], np.int32), np.array([0.5], np.float32)), None),
          qb.submit_arrays(_vec(4), None, {"lecture": 1})]
    assert [f.result(timeout=10)[0].chunk.text for f in fs] == ["1", "2", "3", "4"]
    qb.close()
    seen = {(c[1]["lecture"] if c[1] else None, c[2]): c[0] for c in fr.calls}
    assert seen == {(1, False): 2, (None, False): 1, (None, True): 1}


def test_failures_reach_every_caller_and_close_is_final():
    from audio_rag_amd.retrieval.batcher import QueryBatcher

    qb = QueryBatcher(FakeRetriever(fail=True), max_wait_ms=20.0)
    fs = [qb.submit_arrays(_vec(i)) for i in range(5)]
    for f in fs:
        with pytest.raises(RetrievalError, match="device lost"):
            f.result(timeout=10)
    qb.close()
    with pytest.raises(RetrievalError, match="closed"):
        qb.submit_arrays(_vec(1))


def test_sparse_terms_sorted_and_validated():
    import numpy as np

    from audio_rag_amd.core.exceptions import RetrievalError
    from audio_rag_amd.retrieval.batcher import _sorted_csr, _sorted_terms

    idx, val = _sorted_terms([9, 3, 7], [0.9, 0.3, 0.7])
    assert idx.tolist() == [3, 7, 9] and idx.dtype == np.int32
    assert np.allclose(val, [0.3, 0.7, 0.9])
    with pytest.raises(RetrievalError):
        _sorted_terms([4, 4], [1.0, 2.0])
    p, i, v = _sorted_csr([0, 3, 3, 5], [8, 2, 5, 1, 0], [8.0, 2.0, 5.0, 1.0, 0.0])
    assert p.tolist() == [0, 3, 3, 5] and i.tolist() == [2, 5, 8, 0, 1]
    assert v.tolist() == [2.0, 5.0, 8.0, 0.0, 1.0]
    with pytest.raises(RetrievalError):
        _sorted_csr([0, 2], [6, 6], [1.0, 1.0])
