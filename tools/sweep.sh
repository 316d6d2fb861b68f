#!/bin/bash
# N=1 corpus-size sweep (north_star: 10k / 100k / 1M / 10M chunks) for the dense and hybrid
# workloads; one JSON line per run in gpurun_out/${TAG}_<workload>_<chunks>.log
TAG=${1:-sw}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for w in dense hybrid; do
  for n in 10000 100000 1000000 10000000; do
    timeout -k 10 400 python bench.py --workload $w --chunks $n --steps 30 --warmup 5 --no-cpu-baseline \
      > gpurun_out/${TAG}_${w}_${n}.log 2>&1 || { echo "$w $n failed rc=$?"; exit 1; }
    echo "$w $n $(tail -1 gpurun_out/${TAG}_${w}_${n}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), "qps", round(d["ms_per_step"],3), "ms/step p50", round(d["p50_ms"],3), "single", round(d["p50_single_query_ms"],3), "scan_frac", round(d["roofline"]["frac"],3))')"
  done
done
