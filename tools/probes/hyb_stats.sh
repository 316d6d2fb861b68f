#!/bin/bash
# Kernel-trace statistics of the hybrid step (bench.py --workload hybrid, configs[2]'s retrieval).
TAG=${1:-hybst}
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
P="$R/gpurun_out/${TAG}_p"; mkdir -p "$P"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$P/hyb" -o run -- python3 $R/bench.py --workload hybrid --steps 20 --warmup 3 --no-cpu-baseline --no-extras --latency-iters 2 > "$P/hyb.log" 2>&1 || exit $?
python3 "$R/tools/rocpd_stats.py" "$P/hyb/run_results.db" > "$R/gpurun_out/${TAG}_hybrid_kernel_stats.csv" || exit $?
python3 "$R/tools/rocpd_timeline.py" "$P/hyb/run_results.db" 400 > "$R/gpurun_out/${TAG}_hybrid_timeline.csv" || exit $?
rm -rf "$P"
head -25 "$R/gpurun_out/${TAG}_hybrid_kernel_stats.csv" | cut -c1-160
head -3 "$R/gpurun_out/${TAG}_hybrid_timeline.csv"
