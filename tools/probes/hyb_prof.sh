#!/bin/bash
# Kernel stats of the hybrid bench (1M rows, 64 queries per step) under rocprofv3 --kernel-trace.
TAG=${1:-hybp}
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp; mkdir -p "$R/gpurun_out"
P=/tmp/${TAG}_prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P -o run -- python3 $R/bench.py --workload hybrid --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 1 > "$R/gpurun_out/${TAG}.log" 2>&1 || exit 1
python3 "$R/tools/rocpd_stats.py" $P/run_results.db > "$R/gpurun_out/${TAG}_kernel_stats.csv" || exit 1
tail -1 "$R/gpurun_out/${TAG}.log" | cut -c1-200
cut -c1-160 "$R/gpurun_out/${TAG}_kernel_stats.csv" | head -16
