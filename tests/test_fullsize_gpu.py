"""Parity at BASELINE.json's full sizes, on the GPU, against the CPU oracle.

configs[2] (1 x MI355X, 1M chunks, hybrid dense + BM25 with RRF, top-20 -> cross-encoder -> 5):
  * MI355XRetriever.search_batch in hybrid mode over 1M x 1024 fp16 rows + the SURVEY §8(d) Zipf
    sparse corpus: prefetch 40 + 40 -> RRF 20 (qdrant.py:281-298). The dense and sparse prefetch
    lists and the fused ids / fp64 RRF scores must equal the oracle's bit for bit.
  * the cross-encoder (reranking/bge.py:86-147) on the top-20 candidates of 16 queries (320 pairs
    of L = 256 tokens, all 12 layers, fp16 path) within 1e-3 of transformers' fp32 forward.
configs[3]'s arithmetic on one GPU (10M chunks sharded 8-way -> 8 shards of 1.25M rows, the
all-gathered batch of 512 queries, i.e. exactly one rank's scan shape at N = 8):
  * per-shard tiled scans (dense_gemm_scan_w4_kernel, the default tiled form) at k = 5 and k = 40, merged over the 8
    shards by armi_topk_merge_shards: 8 sampled queries against the oracle over all 10M rows,
    all 512 against the exhaustive exact scan;
  * the hybrid step: dense + sparse prefetch 40 per shard, merged, RRF 20, against the oracle.
The inputs come from audio_rag_amd.synthetic (seeded, generated on the device); the oracle reads
host copies of the same bytes.
"""

import numpy as np
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

N1 = 1_000_000
SHARDS, SHARD_ROWS = 8, 1_250_000
DIM = 1024


def _host_csr(indptr, idx, val):
    return indptr.cpu().numpy(), idx.cpu().numpy(), val.cpu().numpy()


def _rows_u16(t: torch.Tensor) -> np.ndarray:
    return t.cpu().numpy().view(np.uint16)


def _assert_dense_equal(got, want, q_sel=None):
    """ids, exact keys and scores of a device TopK against an oracle TopK (rows q_sel)."""
    sel = slice(None) if q_sel is None else q_sel
    ids = got.ids.cpu().numpy()[sel]
    np.testing.assert_array_equal(ids, want.ids)
    np.testing.assert_array_equal(got.count.cpu().numpy()[sel], want.count)
    live = want.ids >= 0
    np.testing.assert_array_equal(got.rank.cpu().numpy()[sel][live], want.rank[live])
    np.testing.assert_array_equal(got.scores.cpu().numpy()[sel][live], want.scores[live])


def _assert_sparse_equal(got, want, q_sel=None):
    sel = slice(None) if q_sel is None else q_sel
    cnt = got.count.cpu().numpy()[sel]
    np.testing.assert_array_equal(cnt, want.count)
    ids = got.ids.cpu().numpy()[sel]
    sc = got.scores.cpu().numpy()[sel]
    for q in range(len(cnt)):
        c = int(cnt[q])
        np.testing.assert_array_equal(ids[q, :c], want.ids[q, :c])
        np.testing.assert_array_equal(sc[q, :c], want.scores[q, :c])


def _assert_rrf_equal(o, fused, d_ids, d_cnt, s_ids, s_cnt, limit, q_sel=None):
    """fused device TopK (ids + fp64 RRF score) against qdrant-client local-mode RRF of the
    oracle's prefetch lists."""
    ids = fused.ids.cpu().numpy()
    rank = fused.rank.cpu().numpy()
    cnt = fused.count.cpu().numpy()
    rows = range(len(d_cnt)) if q_sel is None else q_sel
    for j, q in enumerate(rows):
        want = o.rrf([[int(x) for x in d_ids[j, :d_cnt[j]]], [int(x) for x in s_ids[j, :s_cnt[j]]]],
                     limit)
        assert int(cnt[q]) == len(want)
        assert [int(x) for x in ids[q, :len(want)]] == [p for p, _ in want]
        assert [float(x) for x in rank[q, :len(want)]] == [v for _, v in want]


# ----------------------------------------------------------------------------- configs[2]

@pytest.fixture(scope="module")
def corpus_1m(gpu):
    from audio_rag_amd.synthetic import (VOCAB, make_queries, make_rows, make_sparse_queries,
                                         make_sparse_rows)

    rows = make_rows(0, N1, DIM, gpu)
    csr = make_sparse_rows(0, N1, gpu)
    q = make_queries(1, 16, DIM, gpu, seed=11)[0].contiguous()
    qcsr = make_sparse_queries(16, gpu, seed=12)
    torch.cuda.synchronize()
    return dict(rows=rows, csr=csr, q=q, qcsr=qcsr, vocab=VOCAB)


def test_configs2_hybrid_1m_matches_oracle(corpus_1m, oracle_mod):
    from audio_rag_amd.config import RetrievalConfig
    from audio_rag_amd.retrieval.collection import ChunkCollection
    from audio_rag_amd.retrieval.device import DenseIndex, SparseIndex
    from audio_rag_amd.retrieval.mi355x import MI355XRetriever, QueryBatch

    o = oracle_mod
    c = corpus_1m
    dense = DenseIndex(c["rows"])
    sparse = SparseIndex(*c["csr"], vocab=c["vocab"])
    ret = MI355XRetriever(RetrievalConfig(), DIM)
    ret.attach_collection(ChunkCollection.from_indexes("audio_rag", dense, [{}] * N1, sparse))
    qi, qx, qv = c["qcsr"]
    fused, mode = ret.search_batch(QueryBatch(dense=c["q"], sparse_indptr=qi, sparse_indices=qx,
                                              sparse_values=qv), top_k=20, search_type="hybrid")
    d40 = dense.topk(c["q"], 40)
    s40 = sparse.topk(qi, qx, qv, 40)
    torch.cuda.synchronize()
    assert mode == "hybrid"
    assert bool((d40.flags == 1).all())  # the fast path certified every query at 1M

    rows = _rows_u16(c["rows"])
    q16 = _rows_u16(c["q"])
    hcsr = _host_csr(*c["csr"])
    qh = _host_csr(qi, qx, qv)
    want_d = o.dense_topk(rows, q16, 40)
    want_s = o.sparse_topk(*hcsr, *qh, 40)
    _assert_dense_equal(d40, want_d)
    _assert_sparse_equal(s40, want_s)
    _assert_rrf_equal(o, fused, want_d.ids, want_d.count, want_s.ids, want_s.count, 20)
    assert int(fused.count.min()) == 20


def test_configs2_rerank_full_depth_within_1e3(corpus_1m, gpu):
    """Cross-encoder over the retrieved top-20 of all 16 queries: 320 (query, chunk) pairs of 256
    tokens (<s> q16 </s></s> d236 </s>, bench.py's pair layout) through all 12 layers (fp16 GEMMs /
    attention, the graphed forward) against transformers' fp32 forward of the same seeded weights
    (round 5: 16 queries, was 2)."""
    from audio_rag_amd.reranking.xlmr import CrossEncoderXLMR, build_reranker
    from audio_rag_amd.retrieval.device import DenseIndex
    from audio_rag_amd.synthetic import VOCAB, doc_tokens

    c = corpus_1m
    nq = c["q"].shape[0]
    cand = DenseIndex(c["rows"]).topk(c["q"], 20).ids  # [nq, 20] ordinals
    g = torch.Generator(device=gpu).manual_seed(4)
    q_tok = torch.randint(4, VOCAB, (nq, 16), generator=g, device=gpu, dtype=torch.int32)
    docs = doc_tokens(cand, 236)
    eos = torch.full((nq, 20, 1), 2, dtype=torch.int32, device=gpu)
    bos = torch.zeros((nq, 20, 1), dtype=torch.int32, device=gpu)
    pairs = torch.cat([bos, q_tok[:, None, :].expand(nq, 20, 16), eos, eos, docs, eos],
                      dim=2).reshape(nq * 20, 256).contiguous()
    mask = torch.ones_like(pairs)
    model = build_reranker(seed=5)
    enc = CrossEncoderXLMR(model, gpu)
    enc.to_dtype(torch.float16)
    got = enc.forward(pairs, mask).cpu().numpy().astype(np.float64)
    want = []
    with torch.no_grad():
        for b in range(0, nq * 20, 40):
            ids = pairs[b:b + 40].long().cpu()
            want.append(torch.sigmoid(model(input_ids=ids, attention_mask=torch.ones_like(ids)
                                            ).logits.double()).view(-1).numpy())
    want = np.concatenate(want)
    err = np.abs(got - want).max()
    print(f"configs[2] rerank {nq * 20} pairs x 256 tokens, 12 layers: "
          f"max |score error| = {err:.2e}")
    assert err < 1e-3
    # the reranked order the pipeline would return (stable sort, reranking/bge.py:134)
    for qq in range(nq):
        o_got = np.argsort(-got[qq * 20:(qq + 1) * 20], kind="stable")[:5]
        o_want = np.argsort(-want[qq * 20:(qq + 1) * 20], kind="stable")[:5]
        gap = np.sort(want[qq * 20:(qq + 1) * 20])[::-1]
        if np.min(np.abs(np.diff(gap[:6]))) > 2e-3:  # order is only defined outside the budget
            assert list(o_got) == list(o_want)


# ----------------------------------------------------------------------------- configs[3]

@pytest.fixture(scope="module")
def shards_10m(gpu):
    from audio_rag_amd.retrieval.device import DenseIndex
    from audio_rag_amd.synthetic import make_queries, make_rows

    idx = []
    for s in range(SHARDS):
        rows = make_rows(s * SHARD_ROWS, SHARD_ROWS, DIM, gpu)
        idx.append(DenseIndex(rows, ordinal_base=s * SHARD_ROWS))
    q = make_queries(1, 512, DIM, gpu, seed=21)[0].contiguous()
    torch.cuda.synchronize()
    yield dict(idx=idx, q=q)
    for ix in idx:
        ix.close()
    torch.cuda.empty_cache()


def _host_rows_10m(shards):
    out = np.empty((SHARDS * SHARD_ROWS, DIM), dtype=np.uint16)
    for s, ix in enumerate(shards["idx"]):
        out[s * SHARD_ROWS:(s + 1) * SHARD_ROWS] = _rows_u16(ix.rows)
    return out


def _merge(lists, k):
    from audio_rag_amd.retrieval.device import merge_shards

    st = lambda name: torch.stack([getattr(t, name) for t in lists])
    return merge_shards(st("rank"), st("scores"), st("ids"), st("count"), k)


SAMPLE = [0, 1, 63, 64, 255, 256, 400, 511]


@pytest.mark.parametrize("k", [5, 40])
def test_configs3_shard_scan_512q_matches_oracle_and_exact(shards_10m, oracle_mod, k):
    sh = shards_10m
    q = sh["q"]
    fast = [ix.topk(q, k) for ix in sh["idx"]]
    exact = [ix.topk(q, k, exact=True) for ix in sh["idx"]]
    gf = _merge(fast, k)
    ge = _merge(exact, k)
    torch.cuda.synchronize()
    cert = torch.stack([t.flags for t in fast]).eq(1).float().mean().item()
    print(f"configs[3] per-rank scan 1.25M x 512, k={k}: certified fraction {cert:.4f}")
    # all 512 queries: the tiled fast path (certified or re-run exactly) == exhaustive exact scan
    np.testing.assert_array_equal(gf.ids.cpu().numpy(), ge.ids.cpu().numpy())
    np.testing.assert_array_equal(gf.rank.cpu().numpy(), ge.rank.cpu().numpy())
    np.testing.assert_array_equal(gf.scores.cpu().numpy(), ge.scores.cpu().numpy())
    # sampled queries against the oracle over all 10M rows
    rows = sh.get("host")
    if rows is None:
        rows = sh["host"] = _host_rows_10m(sh)
    want = oracle_mod.dense_topk(rows, _rows_u16(q)[SAMPLE], k)
    _assert_dense_equal(gf, want, SAMPLE)


def test_configs3_hybrid_shards_match_oracle(shards_10m, oracle_mod, gpu):
    """The hybrid step of one rank at N = 8: per-shard dense + sparse prefetch 40 for all 512
    all-gathered queries, merged over the 8 shards, RRF 20 (what ShardedSearch.hybrid computes
    around its collectives), against the oracle over the 10M-row corpus."""
    from audio_rag_amd.retrieval.device import SparseIndex, rrf_fuse
    from audio_rag_amd.synthetic import VOCAB, make_sparse_queries, make_sparse_rows

    sh = shards_10m
    q = sh["q"]
    qcsr = make_sparse_queries(512, gpu, seed=22)
    s_lists, csrs = [], []
    for s in range(SHARDS):
        csr = make_sparse_rows(s * SHARD_ROWS, SHARD_ROWS, gpu)
        six = SparseIndex(*csr, vocab=VOCAB, ordinal_base=s * SHARD_ROWS)
        s_lists.append(six.topk(*qcsr, 40))
        csrs.append(_host_csr(*csr))
        del csr
    d = _merge([ix.topk(q, 40) for ix in sh["idx"]], 40)
    sp = _merge(s_lists, 40)
    fused = rrf_fuse(d, sp, 20)
    torch.cuda.synchronize()

    o = oracle_mod
    rows = sh.get("host")
    if rows is None:
        rows = sh["host"] = _host_rows_10m(sh)
    nnz = [int(c[0][-1]) for c in csrs]
    indptr = np.zeros(SHARDS * SHARD_ROWS + 1, dtype=np.int64)
    base = 0
    for s, c in enumerate(csrs):
        indptr[s * SHARD_ROWS + 1:(s + 1) * SHARD_ROWS + 1] = c[0][1:] + base
        base += nnz[s]
    indices = np.concatenate([c[1] for c in csrs])
    values = np.concatenate([c[2] for c in csrs])
    qi, qx, qv = _host_csr(*qcsr)
    sel_ptr = np.concatenate([[0], np.cumsum([qi[i + 1] - qi[i] for i in SAMPLE])]).astype(np.int32)
    sel_idx = np.concatenate([qx[qi[i]:qi[i + 1]] for i in SAMPLE]).astype(np.int32)
    sel_val = np.concatenate([qv[qi[i]:qi[i + 1]] for i in SAMPLE]).astype(np.float32)
    want_d = o.dense_topk(rows, _rows_u16(q)[SAMPLE], 40)
    want_s = o.sparse_topk(indptr, indices, values, sel_ptr, sel_idx, sel_val, 40)
    _assert_dense_equal(d, want_d, SAMPLE)
    _assert_sparse_equal(sp, want_s, SAMPLE)
    _assert_rrf_equal(o, fused, want_d.ids, want_d.count, want_s.ids, want_s.count, 20, SAMPLE)


# ------------------------------------------------------------------------------- BGE-M3

def test_bge_m3_full_depth_matches_fp32(gpu):
    """The shipped 24-layer XLM-R-large BGE-M3 forward (fp16 on the GPU, eager and HIP-graph
    replay) against transformers' fp32 CPU forward of the same seeded weights, 4 queries
    (embeddings/bge.py:48-55, 137-157): dense cosine >= 0.999, clear lexical weights within
    tolerance."""
    from audio_rag_amd.config import EmbeddingConfig
    from audio_rag_amd.embeddings.bge_m3 import BGEM3Embedder, build_bge_m3, lexical_weights

    e = BGEM3Embedder(EmbeddingConfig(), device=gpu)
    e.load()
    model, sparse = build_bge_m3(0)
    texts = ["what does the lecturer say about gradient descent",
             "explain the bias variance trade off in the second lecture",
             "kernel",
             "how is the learning rate schedule chosen for the convex objective in the support "
             "vector machine example and why does the professor prefer boosting trees"]
    pairs = []  # (name, fp32 reference vector, GPU vector) for the retrieval bound below
    for text in texts:
        ids = e.tokenizer.encode(text)
        with torch.no_grad():
            h = model(input_ids=torch.tensor([ids])).last_hidden_state
            ref = torch.nn.functional.normalize(h[:, 0], dim=-1)[0].numpy()
            ref_lex = lexical_weights(torch.relu(sparse(h)).squeeze(-1)[0].tolist(), ids)
        for name, (dv, lex) in (("eager", e.encode_ids([ids])), ("graph", e.encode_query_ids(ids))):
            d = dv[0].float().cpu().numpy()
            cos = float(np.dot(ref, d) / np.linalg.norm(d))
            print(f"bge-m3 24 layers {name} L={len(ids)}: cos {cos:.6f}")
            assert cos >= 0.999, (name, cos)
            pairs.append((name, ref, d))
            got = lex[0]
            clear = [t for t, w in ref_lex.items() if w > 0.05]
            assert all(t in got for t in clear), name
            # (the seeded stand-in's sparse head leaves no positive weight on these texts, so
            # this check is empty here; tests/test_lexical_weights_gpu.py compares 34 nonzero
            # weights through a re-biased head)
            np.testing.assert_allclose([got[t] for t in clear], [ref_lex[t] for t in clear],
                                       rtol=5e-2, atol=5e-3)
    _check_encode_error_bounds_topk(pairs, gpu)


def _check_encode_error_bounds_topk(pairs, gpu, n_rows=200_000, k=10):
    """How far the fp16 encode error can move dense top-k ids (retrieval/qdrant.py:281-332 after
    embeddings/bge.py:137-157): with q the GPU vector rounded to fp16 and normalised, and r the fp32
    reference, every row's cosine moves by at most eps = ||q - r|| (unit rows, Cauchy-Schwarz), so
    a row may enter or leave the top-k only when its reference score is within 2 eps of the k-th.
    Over a seeded corpus with 48 rows planted at cosines 0.90-0.99 around each reference (near-ties
    at the top), the GPU top-k of q is checked against that bound; the fraction of ids shared with
    the reference top-k is printed."""
    from audio_rag_amd.retrieval.device import DenseIndex
    from audio_rag_amd.synthetic import make_rows

    base = make_rows(0, n_rows, DIM, gpu)
    g = torch.Generator(device=gpu).manual_seed(11)
    planted = []
    for _, ref, _ in pairs[::2]:  # one reference per text (eager and graph share it)
        r = torch.from_numpy(ref).to(gpu, torch.float32)
        noise = torch.randn((48, DIM), generator=g, device=gpu)
        noise -= (noise @ r)[:, None] * r[None, :]
        noise /= noise.norm(dim=1, keepdim=True)
        c = torch.linspace(0.90, 0.99, 48, device=gpu)[:, None]
        planted.append((c * r[None, :] + torch.sqrt(1 - c * c) * noise).half())
    rows = torch.cat([base] + planted)
    perm = torch.randperm(rows.shape[0], generator=g, device=gpu)
    rows = rows[perm].contiguous()
    idx = DenseIndex(rows)
    r64 = rows.double()
    r64 /= r64.norm(dim=1, keepdim=True)
    shared = []
    for name, ref, d in pairs:
        q16 = torch.from_numpy(d).to(gpu).half()
        q = q16.double() / q16.double().norm()
        r = torch.from_numpy(ref).to(gpu, torch.float64)
        eps = float((q - r).norm())
        s_ref = r64 @ r
        want = torch.argsort(-s_ref, stable=True)[:k]  # ties by ordinal
        out = idx.topk(q16[None, :], k)
        got = out.ids[0].cpu()
        assert int(out.count[0]) == k
        kth = float(s_ref[want[-1]])
        extra = set(got.tolist()) - set(want.cpu().tolist())
        for i in extra:
            assert kth - float(s_ref[i]) <= 2 * eps + 1e-12, (name, i, kth, float(s_ref[i]), eps)
        shared.append(1 - len(extra) / k)
        print(f"bge-m3 {name}: eps {eps:.2e}, top-{k} ids shared with the fp32 encode "
              f"{shared[-1]:.2f} (ref gap k-th to k+1-th "
              f"{kth - float(s_ref[torch.argsort(-s_ref, stable=True)[k]]):.2e})")

