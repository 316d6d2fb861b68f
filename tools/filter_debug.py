"""Why a sparse query is not certified by the MFMA filter: for every query of the sparse_bench
batches that the filter left to the exact scan, the exact scores and the filter's upper-bound
keys of all rows (a numpy / scipy restatement of sparse_filter.h's quantisation), the number of
rows whose key reaches the k-th exact score (the filter needs it <= kc) and the members count.

python tools/filter_debug.py [--rows N] [--k K]"""
import argparse
import os
import sys

import numpy as np
import scipy.sparse as sps
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from audio_rag_amd.retrieval.device import SparseIndex  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--k", type=int, default=40)
    ap.add_argument("--batches", type=int, default=8)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    ip, ix, iv = bench.make_sparse_rows(0, a.rows, dev)
    si = SparseIndex(ip, ix, iv, bench.VOCAB)
    ipn, ixn, ivn = ip.cpu().numpy(), ix.cpu().numpy(), iv.cpu().numpy()
    X = sps.csr_matrix((ivn.astype(np.float64), ixn, ipn), shape=(a.rows, bench.VOCAB))
    tmax = np.zeros(bench.VOCAB, np.float32)
    np.maximum.at(tmax, ixn, ivn)
    s = (tmax / np.float32(255)).astype(np.float32)
    a8 = np.ceil(ivn / np.maximum(s[ixn], 1e-30))
    A = sps.csr_matrix((a8, ixn, ipn), shape=(a.rows, bench.VOCAB))
    kc = max(a.k + 32, 2 * a.k)
    bad = 0
    for b in range(a.batches):
        qi, qx, qv = bench.make_sparse_queries(64, dev, seed=100 + b)
        out = si.topk(qi, qx, qv, a.k)
        fl = out.flags.cpu().numpy()
        qin, qxn, qvn = qi.cpu().numpy(), qx.cpu().numpy(), qv.cpu().numpy()
        for q in np.nonzero((fl & 4) == 0)[0]:
            bad += 1
            t, w = qxn[qin[q]:qin[q + 1]], qvn[qin[q]:qin[q + 1]]
            wq = np.zeros(bench.VOCAB)
            wq[t] = w
            ex = X @ wq
            member = np.asarray((X[:, t] != 0).sum(axis=1)).ravel() > 0
            bq = np.zeros(bench.VOCAB)
            bq[t] = w.astype(np.float64) * s[t]
            key = (A @ bq) * (1 + 2 ** -12)
            kth = np.sort(ex[member])[::-1][a.k - 1] if member.sum() >= a.k else -1
            above = int((key >= kth).sum())
            df = np.asarray((X[:, t] != 0).sum(axis=0)).ravel()
            print(f"batch {b} query {q}: flags {fl[q]} terms {t.size} members {member.sum()} "
                  f"kth {kth:.6f} rows with key >= kth {above} (kc {kc}) "
                  f"df {sorted(df.tolist())}", flush=True)
    print(f"{bad} uncertified of {64 * a.batches}", flush=True)


if __name__ == "__main__":
    main()
