"""One-screen summary of a bench.py JSON line (the default run's headline and child objects).
Usage: python tools/bench_summary.py BENCH_JSON"""
import json
import sys


def main() -> None:
    d = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1])
    r = d["roofline"]
    print(f"dense {d['value']:.0f} q/s {d['ms_per_step']:.4f} ms/step frac {r['frac']:.3f} "
          f"scan {r['avg_launch_ms']:.4f} ms p50 {d.get('p50_ms')}")
    for k in ("configs1", "configs2", "chunks_10k", "chunks_10M", "hybrid", "pipeline",
              "configs3_rank"):
        v = d.get(k)
        if not isinstance(v, dict):
            print(k, v)
            continue
        rr = v.get("roofline") or {}
        print(f"{k}: value {v.get('value')} ms/step {v.get('ms_per_step')} frac {rr.get('frac')} "
              f"avg {rr.get('avg_launch_ms', rr.get('avg_forward_ms'))}")
        for kk in ("roofline_sparse", "sparse_stage", "stage_p50_ms", "roofline_scan"):
            if kk in v:
                print("   ", kk, {a: b for a, b in v[kk].items() if a not in ("note", "kernel")})


if __name__ == "__main__":
    main()
