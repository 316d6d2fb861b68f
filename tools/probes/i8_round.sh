#!/bin/bash
# Int8-filter dense path: bench lines (dense with cpu_baseline, hybrid), rocprofv3 kernel stats
# of the dense bench, FETCH_SIZE / WRITE_SIZE passes of dense_scan_i8_kernel.
TAG=${1:-r02i}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench_dense.log 2>&1 || exit $?
echo "dense: $(tail -1 gpurun_out/${TAG}_bench_dense.log | cut -c1-240)"
timeout -k 10 600 python bench.py --workload hybrid > gpurun_out/${TAG}_bench_hybrid.log 2>&1 || exit $?
echo "hybrid: $(tail -1 gpurun_out/${TAG}_bench_hybrid.log | cut -c1-160)"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --latency-iters 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof" -o run -- python3 $B > "$R/gpurun_out/${TAG}_prof.log" 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/${TAG}_fetch" -o run -- python3 $B > "$R/gpurun_out/${TAG}_fetch.log" 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/${TAG}_write" -o run -- python3 $B > "$R/gpurun_out/${TAG}_write.log" 2>&1 || exit $?
echo "pmc done"
