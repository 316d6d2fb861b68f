"""Dense cosine top-k on the GPU (armi_dense_topk) against the CPU oracle.

Parity bar (integer / index work): ids, counts and the float64 ranking key must be bit-identical
to oracle.dense_topk; scores are the float32 cast of key * inv_q on both sides, also bitwise.
Reference call sites: src/audio_rag/retrieval/qdrant.py:284-288 (dense prefetch) and 316-332.
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev(a, gpu):
    return torch.from_numpy(np.ascontiguousarray(a)).to(gpu)


def _index(rows_u16, gpu, base=0):
    from audio_rag_amd.retrieval.device import DenseIndex

    t = _dev(rows_u16.view(np.float16), gpu)
    return DenseIndex(t, ordinal_base=base)


def _run(idx, q_u16, k, gpu, mask=None, exact=False):
    q = _dev(q_u16.view(np.float16), gpu)
    m = None if mask is None else _dev(mask.view(np.int64), gpu)
    out = idx.topk(q, k, row_mask=m, exact=exact)
    torch.cuda.synchronize()
    return {f: getattr(out, f).cpu().numpy() for f in ("ids", "scores", "rank", "count", "flags")}


def _assert_same(got, ref, k):
    np.testing.assert_array_equal(got["count"], ref.count)
    for b in range(ref.count.shape[0]):
        c = ref.count[b]
        np.testing.assert_array_equal(got["ids"][b, :c], ref.ids[b, :c], err_msg=f"query {b}")
        np.testing.assert_array_equal(got["rank"][b, :c], ref.rank[b, :c], err_msg=f"query {b}")
        np.testing.assert_array_equal(got["scores"][b, :c], ref.scores[b, :c], err_msg=f"query {b}")
        assert (got["ids"][b, c:] == -1).all()


@pytest.mark.parametrize("dim", [256, 1024])
def test_norms_bitwise(gpu, oracle_mod, dim):
    rows = oracle_mod.unit_fp16(777, dim, seed=3)
    idx = _index(rows, gpu)
    n2, inv, inv32 = (t.cpu().numpy() for t in idx.norms())
    o2, oinv = oracle_mod.row_norms(rows, dim)
    np.testing.assert_array_equal(n2, o2)
    np.testing.assert_array_equal(inv, oinv)  # GPU f64 sqrt/div must round like IEEE
    np.testing.assert_array_equal(inv32, (oinv * 2.0**24).astype(np.float32))


@pytest.mark.parametrize("n,dim,b,k", [
    (1000, 256, 8, 5), (4099, 1024, 16, 5), (20000, 1024, 64, 40), (3001, 512, 70, 20),
    (50, 768, 3, 5), (5, 256, 4, 8), (1, 1024, 2, 5),
    # > 64 queries: the GEMM-tiled multi-block scan (one / two / three 256-query blocks)
    (20000, 1024, 300, 5), (5000, 256, 130, 40), (100, 768, 513, 5), (33, 1024, 600, 7)])
def test_dense_topk_matches_oracle(gpu, oracle_mod, n, dim, b, k):
    rows = oracle_mod.unit_fp16(n, dim, seed=10 + n)
    qs = oracle_mod.unit_fp16(b, dim, seed=11 + n)
    idx = _index(rows, gpu, base=1000)
    ref = oracle_mod.dense_topk(rows, qs, k, ordinal_base=1000)
    for _ in range(2):  # consecutive calls scan in opposite directions
        _assert_same(_run(idx, qs, k, gpu), ref, k)


@pytest.mark.parametrize("b", [63, 64, 65, 128, 129, 256, 257])
def test_batch_size_boundaries(gpu, oracle_mod, b):
    """Query counts at the scan-form boundaries: one 64-query pass, the XCD-grouped multi-block
    scan (65-128), the tiled scan with one / two 256-query blocks."""
    rows = oracle_mod.unit_fp16(3000, 1024, seed=40 + b)
    qs = oracle_mod.unit_fp16(b, 1024, seed=41 + b)
    idx = _index(rows, gpu, base=5)
    _assert_same(_run(idx, qs, 5, gpu), oracle_mod.dense_topk(rows, qs, 5, ordinal_base=5), 5)


@pytest.mark.parametrize("n,b", [(20000, 32), (20000, 200)])
def test_max_k(gpu, oracle_mod, n, b):
    """k = 240 (MAX_K), on the 64-query scan and on the tiled scan."""
    from audio_rag_amd.retrieval.device import MAX_K

    rows = oracle_mod.unit_fp16(n, 1024, seed=50 + b)
    qs = oracle_mod.unit_fp16(b, 1024, seed=51 + b)
    idx = _index(rows, gpu)
    _assert_same(_run(idx, qs, MAX_K, gpu), oracle_mod.dense_topk(rows, qs, MAX_K), MAX_K)


def test_fast_path_certifies(gpu, oracle_mod):
    """The MFMA scan + exact rescore must certify random queries itself (the exact fallback
    would otherwise hide a broken fast path)."""
    rows = oracle_mod.unit_fp16(60000, 1024, seed=5)
    qs = oracle_mod.unit_fp16(64, 1024, seed=6)
    idx = _index(rows, gpu)
    for k in (5, 40):
        got = _run(idx, qs, k, gpu)
        assert (got["flags"] == 1).all(), got["flags"]
        ref = oracle_mod.dense_topk(rows, qs, k)
        _assert_same(got, ref, k)


def test_multi_block_scan_certifies_and_masks(gpu, oracle_mod):
    """512 queries (the all-gathered batch of an 8-GPU step) over one shard: the multi-block
    scan must certify by itself, honour a row mask and equal the oracle."""
    n = 20000
    rows = oracle_mod.unit_fp16(n, 1024, seed=17)
    qs = oracle_mod.unit_fp16(512, 1024, seed=18)
    idx = _index(rows, gpu, base=123)
    got = _run(idx, qs, 5, gpu)
    assert (got["flags"] == 1).all(), np.unique(got["flags"], return_counts=True)
    _assert_same(got, oracle_mod.dense_topk(rows, qs, 5, ordinal_base=123), 5)
    rng = np.random.default_rng(3)
    mask = np.zeros((n + 63) // 64, dtype=np.uint64)
    for r in np.nonzero(rng.random(n) < 0.4)[0]:
        mask[r >> 6] |= np.uint64(1) << np.uint64(r & 63)
    got = _run(idx, qs[:200], 20, gpu, mask=mask)
    _assert_same(got, oracle_mod.dense_topk(rows, qs[:200], 20, row_mask=mask,
                                            ordinal_base=123), 20)


def test_exact_entry_point(gpu, oracle_mod):
    rows = oracle_mod.unit_fp16(9000, 1024, seed=7)
    qs = oracle_mod.unit_fp16(5, 1024, seed=8)
    idx = _index(rows, gpu)
    got = _run(idx, qs, 33, gpu, exact=True)
    _assert_same(got, oracle_mod.dense_topk(rows, qs, 33), 33)


def test_row_mask_and_invalid_rows(gpu, oracle_mod):
    n = 5000
    rows = oracle_mod.unit_fp16(n, 256, seed=9).copy()
    rows[17, 3] = 0x7C00  # +inf: outside the fp16 domain -> never a result
    rows[4000, 0] = 0x4400  # 4.0: |x| >= 2 -> invalid
    qs = oracle_mod.unit_fp16(6, 256, seed=10)
    rng = np.random.default_rng(0)
    bits = rng.random(n) < 0.3
    mask = np.zeros((n + 63) // 64, dtype=np.uint64)
    for r in np.nonzero(bits)[0]:
        mask[r >> 6] |= np.uint64(1) << np.uint64(r & 63)
    idx = _index(rows, gpu)
    assert idx.invalid_rows() == 2
    got = _run(idx, qs, 12, gpu, mask=mask)
    ref = oracle_mod.dense_topk(rows, qs, 12, row_mask=mask)
    _assert_same(got, ref, 12)
    assert not np.isin(got["ids"], [17, 4000]).any()


def test_few_enabled_rows_and_exact_ties(gpu, oracle_mod):
    rows = oracle_mod.unit_fp16(3000, 1024, seed=12).copy()
    rows[100:140] = rows[7]  # 41 identical rows: exact key ties broken by ordinal
    qs = np.vstack([rows[7], oracle_mod.unit_fp16(3, 1024, seed=13)])
    idx = _index(rows, gpu)
    got = _run(idx, qs, 45, gpu)
    ref = oracle_mod.dense_topk(rows, qs, 45)
    _assert_same(got, ref, 45)
    mask = np.zeros((3000 + 63) // 64, dtype=np.uint64)
    mask[0] = np.uint64(0b1011)  # 3 rows enabled, k = 5 -> count 3
    got = _run(idx, qs, 5, gpu, mask=mask)
    ref = oracle_mod.dense_topk(rows, qs, 5, row_mask=mask)
    _assert_same(got, ref, 5)
    assert (got["count"] == 3).all()


def test_zero_query_and_empty_index(gpu, oracle_mod):
    rows = oracle_mod.unit_fp16(500, 256, seed=14)
    qs = np.zeros((2, 256), dtype=np.uint16)
    idx = _index(rows, gpu)
    got = _run(idx, qs, 5, gpu)
    _assert_same(got, oracle_mod.dense_topk(rows, qs, 5), 5)
    empty = _index(np.zeros((0, 256), dtype=np.uint16), gpu)
    got = _run(empty, oracle_mod.unit_fp16(3, 256, seed=1), 5, gpu)
    assert (got["count"] == 0).all()


def test_shard_merge_equals_global(gpu, oracle_mod):
    from audio_rag_amd.retrieval.device import merge_shards

    rows = oracle_mod.unit_fp16(12000, 1024, seed=15)
    qs = oracle_mod.unit_fp16(10, 1024, seed=16)
    k = 20
    parts = []
    for s, (a, b) in enumerate([(0, 3000), (3000, 7001), (7001, 12000)]):
        idx = _index(rows[a:b], gpu, base=a)
        parts.append(idx.topk(_dev(qs.view(np.float16), gpu), k))
    stack = lambda f: torch.stack([getattr(p, f) for p in parts])
    m = merge_shards(stack("rank"), stack("scores"), stack("ids"), stack("count"), k)
    torch.cuda.synchronize()
    got = {f: getattr(m, f).cpu().numpy() for f in ("ids", "scores", "rank", "count")}
    _assert_same(got, oracle_mod.dense_topk(rows, qs, k), k)


@pytest.mark.slow
def test_full_size_fast_equals_exact(gpu, oracle_mod):
    """BASELINE size (1M x 1024): the certified fast path equals the exhaustive exact scan for a
    batch, and both equal the C oracle on two queries."""
    n, dim = 1_000_000, 1024
    g = torch.Generator(device=gpu).manual_seed(0)
    x = torch.randn((n, dim), generator=g, device=gpu)
    rows = (x / x.norm(dim=1, keepdim=True)).half()
    del x
    from audio_rag_amd.retrieval.device import DenseIndex

    idx = DenseIndex(rows)
    qx = torch.randn((64, dim), generator=g, device=gpu)
    q = (qx / qx.norm(dim=1, keepdim=True)).half()
    fast = idx.topk(q, 5)
    exact = idx.topk(q[:4], 5, exact=True)
    torch.cuda.synchronize()
    assert (fast.flags.cpu().numpy() == 1).all()
    np.testing.assert_array_equal(fast.ids[:4].cpu().numpy(), exact.ids.cpu().numpy())
    np.testing.assert_array_equal(fast.rank[:4].cpu().numpy(), exact.rank.cpu().numpy())
    rows_u16 = rows.cpu().numpy().view(np.uint16)
    q_u16 = q[:2].cpu().numpy().view(np.uint16)
    ref = oracle_mod.dense_topk(rows_u16, q_u16, 5)
    np.testing.assert_array_equal(fast.ids[:2].cpu().numpy(), ref.ids)
    np.testing.assert_array_equal(fast.rank[:2].cpu().numpy(), ref.rank)


def test_batches_on_two_streams(gpu, oracle_mod):
    """Batches alternating over two HIP streams with their own workspaces (a serving front end's
    pattern), a row filter on every other batch and one batch whose queries sit on a pile of 100
    exact duplicate rows (more than the 64 rescored: the second pass finds them). Every answer
    equals the oracle's."""
    n = 40000
    rows = oracle_mod.unit_fp16(n, 1024, seed=81)
    rows[1000:1100] = rows[1000]
    idx = _index(rows, gpu)
    streams = [torch.cuda.Stream(device=gpu) for _ in range(2)]
    ws = [torch.empty(idx.workspace_bytes(64, 10), dtype=torch.uint8, device=gpu) for _ in range(2)]
    mask = np.zeros((n + 63) // 64, dtype=np.uint64)
    mask[::3] = np.uint64(0xF0F0F0F0F0F0F0F0)
    m_dev = _dev(mask.view(np.int64), gpu)
    qs = [oracle_mod.unit_fp16(64, 1024, seed=82 + i) for i in range(7)]
    qs[2][:8] = rows[1000]  # queries equal to the duplicated row (an unfiltered batch)
    q_dev = [_dev(q.view(np.float16), gpu) for q in qs]
    torch.cuda.synchronize()
    for st in streams:
        st.wait_stream(torch.cuda.current_stream())
    outs = []
    for i in range(7):
        with torch.cuda.stream(streams[i % 2]):
            outs.append(idx.topk(q_dev[i], 10, row_mask=m_dev if i % 2 else None,
                                 workspace=ws[i % 2]))
    torch.cuda.synchronize()
    for i in range(7):
        ref = oracle_mod.dense_topk(rows, qs[i], 10, row_mask=mask if i % 2 else None)
        got = {f: getattr(outs[i], f).cpu().numpy() for f in ("ids", "scores", "rank", "count")}
        _assert_same(got, ref, 10)
    assert (outs[2].flags[:8].cpu().numpy() != 1).all()  # the duplicate pile: second pass taken


@pytest.mark.parametrize("mode", ["two_stage", "exact"])
@pytest.mark.parametrize("k", [5, 40])
def test_merge_rescore_modes_near_ties(gpu, oracle_mod, monkeypatch, mode, k):
    """dense_merge_kernel's rescore: fp32 keys first, int64 exact keys only within the fp32 error
    of the k-th (ARMI_MERGE_RESCORE=two; the default for kc > 64), or all kc exactly (=exact; the
    default for kc <= 64). Rows that differ from
    each other by one fp16 ulp in one component, exact duplicates around the k-th position and
    a query equal to a row: both modes return the oracle's answer bit for bit."""
    monkeypatch.setenv("ARMI_MERGE_RESCORE", "exact" if mode == "exact" else "two")
    rows = oracle_mod.unit_fp16(30000, 1024, seed=91)
    base = rows[500].copy()
    for j in range(1, 60):  # one-ulp neighbours of row 500 in component j
        r = base.copy()
        r[j] = np.uint16(int(r[j]) + (1 if j % 2 else -1))
        rows[500 + j] = r
    rows[700:712] = rows[500]  # exact duplicates
    idx = _index(rows, gpu)
    qs = oracle_mod.unit_fp16(64, 1024, seed=92)
    qs[:4] = rows[500]
    qs[4:8] = rows[530]
    got = _run(idx, qs, k, gpu)
    _assert_same(got, oracle_mod.dense_topk(rows, qs, k), k)
