#!/bin/bash
# Kernel-trace of the dense step with the live timing off / at period 8: the gaps around the scan.
TAG=${1:-gap}
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
for v in 0 8; do
  for n in 1000000 100000; do
    ARMI_BENCH_TIMING=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_${v}_$n" -o run -- python3 "$R/bench.py" --chunks $n --steps 100 --warmup 10 --no-cpu-baseline --no-extras --latency-iters 2 > "$R/gpurun_out/${TAG}_${v}_$n.log" 2>&1 || exit $?
  done
done
