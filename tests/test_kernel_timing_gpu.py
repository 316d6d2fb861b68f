"""Live kernel timing (armi_scan_timing_enable / armi_kernel_timing_read, what bench.py's roofline
objects divide by): the timed launches carry their events on the dispatch itself
(hipExtLaunchKernel), so a timed call answers exactly as an untimed one, every timed launch is
counted once with a positive duration, a period n times every n-th launch of a slot, a sparse
call times its whole stage or its scan (never both), and nothing is recorded while timing is
off."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _read(lib, slot):
    ms, n = ctypes.c_double(), ctypes.c_int64()
    lib.call("armi_kernel_timing_read", slot, ctypes.byref(ms), ctypes.byref(n))
    return ms.value, n.value


def test_timed_launches_counted_and_results_unchanged(gpu):
    from audio_rag_amd import _armi, synthetic
    from audio_rag_amd.retrieval.device import DenseIndex, SparseIndex

    rows = synthetic.make_rows(0, 50_000, 1024, gpu)
    di = DenseIndex(rows)
    q = synthetic.make_queries(1, 64, 1024, gpu, seed=3)[0]
    si = SparseIndex(*synthetic.make_sparse_rows(0, 50_000, gpu, seed=5), synthetic.VOCAB)
    qs = synthetic.make_sparse_queries(64, gpu, seed=6)
    for slot in (_armi.TIMING_DENSE_SCAN, _armi.TIMING_SPARSE_SCAN, _armi.TIMING_SPARSE_STAGE):
        _read(_armi, slot)
    base_d = di.topk(q, 5)
    base_s = si.topk(*qs, 20)
    torch.cuda.synchronize()
    assert _read(_armi, _armi.TIMING_DENSE_SCAN)[1] == 0  # timing off: nothing recorded
    _armi.call("armi_scan_timing_enable", 1)
    try:
        outs = [(di.topk(q, 5), si.topk(*qs, 20)) for _ in range(3)]
        torch.cuda.synchronize()
        for slot in (_armi.TIMING_DENSE_SCAN, _armi.TIMING_SPARSE_STAGE):
            ms, n = _read(_armi, slot)
            assert n == 3 and ms > 0.0, (slot, n, ms)
        # a call whose whole stage is timed does not also time its scan
        assert _read(_armi, _armi.TIMING_SPARSE_SCAN)[1] == 0
    finally:
        _armi.call("armi_scan_timing_enable", 0)
    # a period of 2: every second launch of each slot is timed
    _armi.call("armi_scan_timing_enable", 2)
    try:
        for _ in range(4):
            di.topk(q, 5)
            si.topk(*qs, 20)
        torch.cuda.synchronize()
        assert _read(_armi, _armi.TIMING_DENSE_SCAN)[1] == 2
        assert _read(_armi, _armi.TIMING_SPARSE_STAGE)[1] == 2  # calls 0 and 2
        ms, n = _read(_armi, _armi.TIMING_SPARSE_SCAN)  # the scans of calls 1 and 3: every 2nd
        assert n == 1 and ms > 0.0
    finally:
        _armi.call("armi_scan_timing_enable", 0)
    for d, s in outs:
        assert torch.equal(d.ids, base_d.ids) and torch.equal(d.scores, base_d.scores)
        assert torch.equal(s.ids, base_s.ids) and torch.equal(s.scores, base_s.scores)
