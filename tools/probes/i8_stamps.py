"""Phase timeline of dense_scan_i8_kernel from a probe build (-DARMI_PROBE_BUILD -DARMI_I8_STAMPS):
per (workgroup, wave) s_memrealtime stamps at entry, after the query image, after the tile loop
and at the end of the workgroup merge, for one 64-query launch over `--chunks` rows. Prints the
launch's phase spans (chip-wide, 10 ns ticks -> us)."""
import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from audio_rag_amd import _armi  # noqa: E402
from audio_rag_amd.retrieval.device import DenseIndex  # noqa: E402
from audio_rag_amd.synthetic import make_queries, make_rows  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rows = make_rows(0, a.chunks, 1024, dev)
    idx = DenseIndex(rows)
    qs = make_queries(1, 64, 1024, dev, seed=1)[0]
    ws = torch.empty(idx.workspace_bytes(64, 5), dtype=torch.uint8, device=dev)
    lib = _armi.load()
    fn = lib.armi_probe_i8_stamps
    fn.argtypes = [ctypes.c_void_p]
    fn.restype = ctypes.c_int
    buf = np.zeros(256 * 8 * 4, dtype=np.uint64)
    mfn = lib.armi_probe_merge_stamps
    mfn.argtypes = [ctypes.c_void_p]
    mfn.restype = ctypes.c_int
    mbuf = np.zeros(64 * 8, dtype=np.uint64)
    mspans = []
    spans = []
    for r in range(a.reps):
        idx.topk(qs, 5, workspace=ws)
        torch.cuda.synchronize()
        assert fn(buf.ctypes.data) == 0
        st = buf.reshape(256, 8, 4).astype(np.int64)
        live = st[:, :, 0] > 0
        t0 = st[:, :, 0][live].min()
        t0_abs = st[:, :, 3][live].max()  # the scan's last workgroup-merge end (absolute ticks)
        rel = (st - t0) / 100.0  # us
        e = rel[..., 0][live]
        img = (rel[..., 1] - rel[..., 0])[live]
        loop = (rel[..., 2] - rel[..., 1])[live]
        merge = (rel[..., 3] - rel[..., 2])[live]
        end = rel[..., 3][live]
        loop_end = rel[..., 2][live]
        le = rel[..., 2]
        xcd_end = [float(np.max(le[x::8][live[x::8]])) if live[x::8].any() else 0.0
                   for x in range(8)]
        # per workgroup (all 8 waves live): the spread of its waves' loop ends and the pure merge
        # (its end minus its last wave's loop end)
        wl = live.all(axis=1)
        wg_spread = (st[wl][:, :, 2].max(axis=1) - st[wl][:, :, 2].min(axis=1)) / 100.0
        wg_merge = (st[wl][:, :, 3].max(axis=1) - st[wl][:, :, 2].max(axis=1)) / 100.0
        wg_end = np.where(live.any(axis=1), np.where(live, rel[..., 2], -1e9).max(axis=1), np.nan)
        wg_loop = np.where(live.any(axis=1), np.where(live, rel[..., 2] - rel[..., 1], np.nan).mean(axis=1), np.nan)
        per_xcd = {}
        for x in range(8):
            ex, lx = wg_end[x::8], wg_loop[x::8]
            ex, lx = ex[~np.isnan(ex)], lx[~np.isnan(lx)]
            if len(ex) > 2:
                ex, lx = np.sort(ex)[1:], lx  # drop the short remainder workgroup
                per_xcd[f"xcd{x}_end_mean"] = float(ex.mean())
                per_xcd[f"xcd{x}_end_max"] = float(ex.max())
                per_xcd[f"xcd{x}_wave_loop_mean"] = float(np.median(lx))
        spans.append(dict(**per_xcd, wg_wave_end_spread_mean=float(wg_spread.mean()),
                          wg_wave_end_spread_max=float(wg_spread.max()),
                          wg_pure_merge_mean=float(wg_merge.mean()),
                          wg_pure_merge_max=float(wg_merge.max()),
                          xcd_loop_end_max_spread=float(max(xcd_end) - min(xcd_end)),
                          entry_spread=float(e.max()), image_mean=float(img.mean()),
                          image_max=float(img.max()), loop_mean=float(loop.mean()),
                          loop_max=float(loop.max()), loop_end_min=float(loop_end.min()),
                          loop_end_max=float(loop_end.max()), merge_mean=float(merge.mean()),
                          merge_max=float(merge.max()), total=float(end.max())))
        buf[:] = 0
        assert mfn(mbuf.ctypes.data) == 0
        ms = mbuf.reshape(64, 8).astype(np.int64)
        ok = (ms > 0).all(axis=1)
        if ok.any():
            m0 = ms[ok][:, 0].min()
            mrel = (ms[ok] - m0) / 100.0
            # per phase: mean duration over the workgroups; start skew; end of the last workgroup
            mspans.append({"start_skew": float(mrel[:, 0].max()),
                           **{f"phase{i}": float(np.mean(mrel[:, i] - mrel[:, i - 1]))
                              for i in range(1, 8)},
                           "total": float(mrel[:, 7].max()),
                           "scan_end_to_merge_start": float((ms[ok][:, 0].min() - t0_abs) / 100.0)})
        mbuf[:] = 0
    keys = spans[0].keys()
    med = {k: float(np.median([s[k] for s in spans[2:]])) for k in keys}
    out = {"chunks": a.chunks, "median_us": med}
    if mspans:
        out["merge_median_us"] = {k: float(np.median([s[k] for s in mspans[2:]]))
                                  for k in mspans[0].keys()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
