"""Seeded synthetic inputs of SURVEY.md §8(d), generated on the device (torch), shared by bench.py
and the full-size parity tests (tests/test_fullsize_gpu.py).

Not part of the query path: the reference ingests real BGE-M3 vectors (embeddings/bge.py:104-157);
these generators stand in for them at BASELINE sizes (1M / 10M chunks), where numpy generation
would take minutes. Every generator is a pure function of (first row, count, seed), chunked in
64k-row blocks with per-block seeds, so a shard's rows are identical whatever the shard count.
"""

from __future__ import annotations

import torch

CHUNK_ROWS = 65536


def make_rows(first: int, count: int, dim: int, device, seed: int = 0) -> torch.Tensor:
    """Rows [first, first+count) of the global synthetic corpus: each 64k-row chunk has its own
    seed, so a shard's rows are identical whatever the shard count."""
    out = torch.empty((count, dim), dtype=torch.float16, device=device)
    c0 = first // CHUNK_ROWS
    c1 = (first + count + CHUNK_ROWS - 1) // CHUNK_ROWS
    for c in range(c0, c1):
        a, b = c * CHUNK_ROWS, (c + 1) * CHUNK_ROWS
        g = torch.Generator(device=device).manual_seed(seed * 1_000_003 + c)
        x = torch.randn((CHUNK_ROWS, dim), generator=g, device=device)
        x = (x / x.norm(dim=1, keepdim=True)).half()
        lo, hi = max(a, first), min(b, first + count)
        if lo < hi:
            out[lo - first:hi - first] = x[lo - a:hi - a]
    return out


def make_queries(n_batches: int, batch: int, dim: int, device, seed: int) -> torch.Tensor:
    g = torch.Generator(device=device).manual_seed(seed)
    x = torch.randn((n_batches, batch, dim), generator=g, device=device)
    return (x / x.norm(dim=2, keepdim=True)).half().contiguous()


# Clustered / anisotropic corpus: what real BGE-M3 chunk vectors of lecture recordings look like
# to the scan, as opposed to the isotropic rows above (VERDICT r02 "the certificate's cliff").
#   * every vector shares one mean direction (weight^2 0.35): random pairs have cosine ~0.35;
#   * a lecture of LECTURE consecutive chunk ordinals shares a topic vector (weight^2 0.20):
#     same-lecture pairs ~0.55;
#   * chunk i's content is the sum of "sentence" vectors u_i .. u_{i+WINDOW-1} (weight^2 0.45):
#     consecutive chunks overlap by WINDOW-1 sentences (the chunker's overlap,
#     src/audio_rag/ingestion/chunking), so neighbours have cosine ~0.89, lag 2 ~0.78;
#   * every DUP_EVERY-th lecture is an exact re-upload of the one before (identical vectors:
#     exact ties, broken by ordinal).
# A query is a noisy mix of three consecutive sentences of a random chunk, so its top hits are a
# contiguous run of near-duplicate ordinals (plus their re-uploaded copies).
LECTURE = 120
WINDOW = 4
DUP_EVERY = 40
_MIX = (0.35 ** 0.5, 0.20 ** 0.5, 0.45 ** 0.5)


def _sentences(block: int, dim: int, device, seed: int) -> torch.Tensor:
    g = torch.Generator(device=device).manual_seed(seed * 1_000_003 + 7919 + block)
    return torch.randn((CHUNK_ROWS + WINDOW, dim), generator=g, device=device) / dim ** 0.5


def _topics(tblock: int, dim: int, device, seed: int) -> torch.Tensor:
    g = torch.Generator(device=device).manual_seed(seed * 1_000_003 + 104729 + tblock)
    return torch.randn((1024, dim), generator=g, device=device) / dim ** 0.5


def _mean_dir(dim: int, device, seed: int) -> torch.Tensor:
    g = torch.Generator(device=device).manual_seed(seed * 1_000_003 + 1)
    v = torch.randn(dim, generator=g, device=device)
    return v / v.norm()


def _clustered(src: torch.Tensor, offsets: tuple, dim: int, device, seed: int) -> torch.Tensor:
    """Unnormalised vectors mean + topic(lecture of src) + sentences src + offsets (fp32)."""
    wa, wb, ws = _MIX
    out = torch.empty((src.numel(), dim), dtype=torch.float32, device=device)
    m = _mean_dir(dim, device, seed)
    blocks = src // CHUNK_ROWS
    for b in torch.unique(blocks).tolist():
        sel = (blocks == b).nonzero().flatten()
        s = src[sel]
        sent = _sentences(b, dim, device, seed)
        loc = s - b * CHUNK_ROWS
        content = sum(sent[loc + o] for o in offsets) / len(offsets) ** 0.5
        del sent
        lect = s // LECTURE
        top = torch.empty_like(content)
        for tb in torch.unique(lect // 1024).tolist():
            ts = (lect // 1024 == tb).nonzero().flatten()
            top[ts] = _topics(tb, dim, device, seed)[lect[ts] - tb * 1024]
        out[sel] = wa * m + wb * top + ws * content
    return out


def make_clustered_rows(first: int, count: int, dim: int, device, seed: int = 3) -> torch.Tensor:
    """Rows [first, first+count) of the global clustered corpus (a pure function of the ordinal,
    so shards agree), L2-normalised fp16."""
    i = torch.arange(first, first + count, device=device, dtype=torch.int64)
    dup = (i // LECTURE) % DUP_EVERY == DUP_EVERY - 1
    src = torch.where(dup, i - LECTURE, i)
    out = torch.empty((count, dim), dtype=torch.float16, device=device)
    step = 4 * CHUNK_ROWS
    for a in range(0, count, step):
        x = _clustered(src[a:a + step], tuple(range(WINDOW)), dim, device, seed)
        out[a:a + step] = (x / x.norm(dim=1, keepdim=True)).half()
    return out


def make_clustered_queries(n: int, n_rows: int, dim: int, device, seed: int,
                           corpus_seed: int = 3, noise: float = 0.3) -> torch.Tensor:
    """n queries, each near a random chunk of the clustered corpus of n_rows rows."""
    g = torch.Generator(device=device).manual_seed(seed)
    p = torch.randint(0, max(n_rows - WINDOW, 1), (n,), generator=g, device=device)
    x = _clustered(p, (1, 2, 3), dim, device, corpus_seed)
    x = x + noise * torch.randn(x.shape, generator=g, device=device) / dim ** 0.5
    return (x / x.norm(dim=1, keepdim=True)).half().contiguous()

VOCAB = 250002


def _zipf_cdf(device, a: float = 1.1) -> torch.Tensor:
    r = torch.arange(1, VOCAB - 4 + 1, dtype=torch.float64, device=device)
    p = r.pow(-a)
    return torch.cumsum(p / p.sum(), 0)


def _sparse_rows(n: int, mean_nnz: float, lo: int, hi: int, wlo: float, whi: float,
                 g: torch.Generator, cdf: torch.Tensor, cap: int):
    """SURVEY §8(d) law on the device: nnz ~ clip(Poisson(mean), lo, hi), unique Zipf(1.1) token
    ids in [4, VOCAB) (sorted per row), weights U(wlo, whi). Returns (counts, indices, values)."""
    dev = cdf.device
    nnz = torch.poisson(torch.full((n,), mean_nnz, device=dev), generator=g).clamp_(lo, hi)
    u = torch.rand((n, cap), generator=g, device=dev, dtype=torch.float64)
    ids = torch.searchsorted(cdf, u).clamp_(max=VOCAB - 5).to(torch.int32) + 4
    ids, _ = torch.sort(ids, dim=1)
    fresh = torch.ones_like(ids, dtype=torch.bool)
    fresh[:, 1:] = ids[:, 1:] != ids[:, :-1]
    rank = torch.cumsum(fresh.to(torch.int32), dim=1)
    keep = fresh & (rank <= nnz[:, None].to(torch.int32))
    counts = keep.sum(dim=1)
    idx = ids[keep]
    vals = torch.empty(idx.numel(), device=dev).uniform_(wlo, whi, generator=g)
    return counts, idx.contiguous(), vals.contiguous()


def make_sparse_rows(first: int, count: int, device, seed: int = 2):
    """CSR rows [first, first+count) of the global synthetic sparse corpus (64k-row chunks with
    their own seeds, as make_rows)."""
    cdf = _zipf_cdf(device)
    cnts, idxs, vals = [], [], []
    c0 = first // CHUNK_ROWS
    c1 = (first + count + CHUNK_ROWS - 1) // CHUNK_ROWS
    for c in range(c0, c1):
        a = c * CHUNK_ROWS
        g = torch.Generator(device=device).manual_seed(seed * 1_000_003 + c)
        cnt, idx, val = _sparse_rows(CHUNK_ROWS, 96.0, 16, 256, 0.01, 0.40, g, cdf, cap=320)
        off = torch.zeros(CHUNK_ROWS + 1, dtype=torch.int64, device=device)
        off[1:] = torch.cumsum(cnt, 0)
        lo, hi = max(a, first) - a, min(a + CHUNK_ROWS, first + count) - a
        if lo < hi:
            cnts.append(cnt[lo:hi])
            idxs.append(idx[off[lo]:off[hi]])
            vals.append(val[off[lo]:off[hi]])
    counts = torch.cat(cnts)
    indptr = torch.zeros(count + 1, dtype=torch.int64, device=device)
    indptr[1:] = torch.cumsum(counts, 0)
    return indptr, torch.cat(idxs).contiguous(), torch.cat(vals).contiguous()


def make_sparse_queries(n: int, device, seed: int):
    g = torch.Generator(device=device).manual_seed(seed)
    cnt, idx, val = _sparse_rows(n, 12.0, 1, 32, 0.05, 0.35, g, _zipf_cdf(device), cap=48)
    indptr = torch.zeros(n + 1, dtype=torch.int32, device=device)
    indptr[1:] = torch.cumsum(cnt, 0).to(torch.int32)
    return indptr, idx, val


def doc_tokens(ordinals: torch.Tensor, length: int) -> torch.Tensor:
    """Synthetic token ids of a chunk (240 tokens, ids in [4, VOCAB)), a pure
    function of the chunk ordinal so every rank can build rerank pairs without a payload table."""
    pos = torch.arange(length, device=ordinals.device, dtype=torch.int64)
    h = ordinals[..., None].to(torch.int64) * 2654435761 + pos * 40503 + 12345
    return (h % (VOCAB - 4) + 4).to(torch.int32)


