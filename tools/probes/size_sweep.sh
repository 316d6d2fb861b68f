#!/bin/bash
# Dense top-5, 64 queries per step, one GPU, at the corpus sizes north_star names (10k, 100k,
# 1M, 10M chunks): q/s, step, first-pass form and its roofline.
TAG=${1:-sz}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
for n in 10000 100000 1000000 10000000; do
  timeout -k 10 400 python bench.py --chunks $n --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 10 > gpurun_out/${TAG}_$n.log 2>&1 || exit $?
  echo "$n: $(tail -1 gpurun_out/${TAG}_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]), round(d["ms_per_step"],4), "p50", round(d["p50_ms"],4), "p50_1q", round(d["p50_single_query_ms"],4), r["kernel"], round(r["avg_launch_ms"],4), round(r["frac"],3), d["certified_frac"])')"
done
