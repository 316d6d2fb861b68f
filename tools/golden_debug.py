"""Replays the golden searches through AudioRAG several times and reports every mismatch with
the raw dense / sparse prefetch lists of the failing search (debug aid)."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "tests" / "golden"))
import replay  # noqa: E402
import test_golden_pipeline_gpu as tg  # noqa: E402
from oracle import oracle as o  # noqa: E402

o.build()
g, s = replay.load()
rag = tg._build(s)
ret = rag.retriever
bad = 0
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    for ci, case in enumerate(g["searches"]):
        q = case["query"]
        mode = o.search_mode(case["search_type"], replay.COLLECTION_HYBRID[case["collection"]], True)
        if mode in ("dense", "legacy_dense"):
            continue
        emb = rag.embedder.embed_query(s["query_texts"][q])
        got = ret.search(emb, top_k=case["top_k"], collection_name=case["collection"],
                         filter_metadata=case["filter"], search_type=case["search_type"])
        got_ids = [r.chunk.metadata["ordinal"] for r in got]
        want_ids = replay.ordinals(case["results"])
        if got_ids != want_ids:
            bad += 1
            coll = ret._collections[case["collection"]]
            qb = ret.to_query_batch([emb])
            mask = coll.filter_mask(case["filter"])
            k2 = 2 * case["top_k"]
            sp = coll.sparse_index.topk(qb.sparse_indptr, qb.sparse_indices, qb.sparse_values, k2,
                                        row_mask=mask)
            torch.cuda.synchronize()
            csr = (coll.sparse_index.indptr.cpu().numpy(), coll.sparse_index.indices.cpu().numpy(),
                   coll.sparse_index.values.cpu().numpy())
            qcsr = (qb.sparse_indptr.cpu().numpy(), qb.sparse_indices.cpu().numpy(),
                    qb.sparse_values.cpu().numpy())
            m = None if mask is None else mask.cpu().numpy().view(np.uint64)
            ref = o.sparse_topk(*csr, *qcsr, k2, row_mask=m)
            print(f"rep {rep} case {ci} coll {case['collection']} mode {mode} k {case['top_k']} "
                  f"filter {case['filter']}\n  got  {got_ids}\n  want {want_ids}\n"
                  f"  sparse gpu {sp.ids[0, :sp.count[0]].tolist()} flags {sp.flags.tolist()}\n"
                  f"  sparse ref {ref.ids[0, :ref.count[0]].tolist()}", flush=True)
print("mismatches", bad)
