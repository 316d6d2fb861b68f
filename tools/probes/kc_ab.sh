#!/bin/bash
# Rows rescored after the int8 pass for k = 10 (hybrid's dense prefetch): kc 128 (default) vs 64.
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
for kc in 128 64 128 64; do
  ARMI_DENSE_KC=$kc timeout -k 10 300 python bench.py --top-k 10 --steps 100 --warmup 5 --no-cpu-baseline --latency-iters 2 > gpurun_out/kc_$kc.log 2>&1 || exit 1
  echo "dense k=10 kc=$kc: $(tail -1 gpurun_out/kc_$kc.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],4), d["certified_frac"])')"
  ARMI_DENSE_KC=$kc timeout -k 10 300 python bench.py --workload hybrid --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 2 > gpurun_out/kch_$kc.log 2>&1 || exit 1
  echo "hybrid kc=$kc: $(tail -1 gpurun_out/kch_$kc.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],4))')"
done
