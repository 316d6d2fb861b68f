"""Corpus sharded by chunk ordinal over the GPUs of one node (one process per GPU).

No reference counterpart: the reference runs a single Qdrant replica
(k8s/helm/audio-rag/values.yaml:137) and scales API processes (Dockerfile.api:85-86). Sharding
is exact for this path because every ranking key is comparable across shards (dense: exact
cosine key; sparse: exact fp32 score; both tie-broken by the global ordinal), so the global top-k
is the top-k of the union of per-shard top-k lists.

One search step for a process group of G ranks, each bringing B queries:
  1. all-gather the queries (RCCL over xGMI): every rank holds all G*B queries
  2. local top-k of all G*B queries on this rank's shard (libarmi kernels)
  3. all-gather the per-shard lists, packed as int64 [G*B, 2k] (key bits, ordinal) and
     int32 [G*B, k+1] (score bits, count): two small collectives
  4. merge this rank's B queries over the G shard lists (armi_topk_merge_shards)
Hybrid search gathers and merges the dense and sparse prefetch lists, then fuses them with RRF.
Per-GPU work is fixed as G grows (shard rows x G*B queries = corpus x B): weak scaling.
"""

from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist

from audio_rag_amd.retrieval.device import TopK

LocalSearch = Callable[[torch.Tensor, int], TopK]
Merge = Callable[[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, int], TopK]


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous ordinal range [lo, hi) owned by `rank` (rank r owns [r*n/G, (r+1)*n/G))."""
    return n * rank // world, n * (rank + 1) // world


def _all_gather(out: torch.Tensor, inp: torch.Tensor, group) -> None:
    """out: [G, *inp.shape]. RCCL gathers straight into the tensor; gloo (CPU tests) into views."""
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, inp, group=group)
    else:
        dist.all_gather(list(out.unbind(0)), inp, group=group)


class ShardedSearch:
    """Sharded top-k over a process group. `local_dense(q, k)` / `local_sparse(qcsr, k)` search
    this rank's shard and return global ordinals; `merge` combines [S, B, k] lists."""

    def __init__(self, local_dense: LocalSearch, merge: Merge, group=None,
                 local_sparse: Callable | None = None, rrf: Callable | None = None):
        self.local_dense = local_dense
        self.local_sparse = local_sparse
        self.merge = merge
        self.rrf = rrf
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def _gather_lists(self, local: TopK, k: int, nb: int) -> TopK:
        """All-gathers per-shard lists of all G*nb queries; merges this rank's nb queries."""
        g = self.world
        dev = local.ids.device
        rank_bits = local.rank.contiguous().view(torch.int64)
        pack_a = torch.cat([rank_bits, local.ids], dim=1).contiguous()                 # [G*nb, 2k]
        pack_b = torch.cat([local.scores.contiguous().view(torch.int32),
                            local.count.view(-1, 1).to(torch.int32)], dim=1).contiguous()  # [G*nb, k+1]
        ga = torch.empty((g,) + tuple(pack_a.shape), dtype=pack_a.dtype, device=dev)
        gb = torch.empty((g,) + tuple(pack_b.shape), dtype=pack_b.dtype, device=dev)
        _all_gather(ga, pack_a, self.group)
        _all_gather(gb, pack_b, self.group)
        mine_a = ga[:, self.rank * nb:(self.rank + 1) * nb]
        mine_b = gb[:, self.rank * nb:(self.rank + 1) * nb]
        return self.merge(mine_a[..., :k].contiguous().view(torch.float64),
                          mine_b[..., :k].contiguous().view(torch.float32),
                          mine_a[..., k:].contiguous(), mine_b[..., k].contiguous(), k)

    def gather_queries(self, q_local: torch.Tensor) -> torch.Tensor:
        out = torch.empty((self.world,) + tuple(q_local.shape), dtype=q_local.dtype,
                          device=q_local.device)
        _all_gather(out, q_local.contiguous(), self.group)
        return out.reshape((-1,) + tuple(q_local.shape[1:]))

    def dense(self, q_local: torch.Tensor, k: int) -> TopK:
        nb = int(q_local.shape[0])
        all_q = self.gather_queries(q_local)
        return self._gather_lists(self.local_dense(all_q, k), k, nb)

    def sparse(self, q_local_csr: tuple[torch.Tensor, torch.Tensor, torch.Tensor], k: int) -> TopK:
        """q_local_csr: (indptr int32 [nb+1], indices int32, values float32) of this rank."""
        indptr, idx, val = q_local_csr
        nb = int(indptr.numel()) - 1
        all_csr = self._gather_csr(indptr, idx, val)
        return self._gather_lists(self.local_sparse(all_csr, k), k, nb)

    def hybrid(self, q_local: torch.Tensor, q_local_csr, k: int) -> TopK:
        """Prefetch dense and sparse 2k each on the global corpus, then RRF(limit=k)."""
        d = self.dense(q_local, 2 * k)
        s = self.sparse(q_local_csr, 2 * k)
        return self.rrf(d, s, k)

    def _gather_csr(self, indptr, idx, val):
        """All-gathers ragged CSR blocks: lengths first, then padded payloads."""
        dev = indptr.device
        n_local = torch.tensor([idx.numel()], dtype=torch.int64, device=dev)
        lens = torch.empty((self.world, 1), dtype=torch.int64, device=dev)
        _all_gather(lens, n_local, self.group)
        lens = lens.view(-1).tolist()
        m = max(max(lens), 1)
        pad_i = torch.zeros(m, dtype=torch.int32, device=dev)
        pad_v = torch.zeros(m, dtype=torch.float32, device=dev)
        pad_i[: idx.numel()] = idx
        pad_v[: val.numel()] = val
        gi = torch.empty((self.world, m), dtype=torch.int32, device=dev)
        gv = torch.empty((self.world, m), dtype=torch.float32, device=dev)
        gp = torch.empty((self.world, indptr.numel()), dtype=torch.int32, device=dev)
        _all_gather(gi, pad_i, self.group)
        _all_gather(gv, pad_v, self.group)
        _all_gather(gp, indptr.to(torch.int32).contiguous(), self.group)
        ptrs, idxs, vals, base = [torch.zeros(1, dtype=torch.int32, device=dev)], [], [], 0
        for r in range(self.world):
            ptrs.append(gp[r, 1:] + base)
            idxs.append(gi[r, : lens[r]])
            vals.append(gv[r, : lens[r]])
            base += lens[r]
        return torch.cat(ptrs), torch.cat(idxs), torch.cat(vals)
