#!/bin/bash
# Kernel-trace stats of the hybrid workload (dense + sparse prefetch, RRF), 1M chunks.
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r01f_prof_hybrid" -o run -- \
  python3 "$R/bench.py" --workload hybrid --steps 10 --warmup 2 --latency-iters 2 --no-cpu-baseline > "$R/gpurun_out/r01f_prof_hybrid.log" 2>&1; rc=$?
echo "prof hybrid rc=$rc"; exit $rc
