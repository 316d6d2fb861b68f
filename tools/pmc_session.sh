#!/bin/bash
# PMC passes for the dense scan kernel (each counter group in its own run, no tracing domains).
TAG=${1:-pmc}
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
B="$R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --latency-iters 2"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/${TAG}_fetch" -o run -- python3 $B > "$R/gpurun_out/${TAG}_fetch.log" 2>&1; rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/${TAG}_write" -o run -- python3 $B > "$R/gpurun_out/${TAG}_write.log" 2>&1; rc=$?; echo "write rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$R/gpurun_out/${TAG}_l2" -o run -- python3 $B > "$R/gpurun_out/${TAG}_l2.log" 2>&1; rc=$?; echo "l2 rc=$rc"
exit $rc
