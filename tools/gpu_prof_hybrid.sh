#!/bin/bash
# Kernel trace of the hybrid workload (1M chunks): tag=$1. rocprofv3 --kernel-trace --stats.
TAG=${1:-hyb}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload hybrid --steps 20 --warmup 3 --no-cpu-baseline --latency-iters 2 ${PROF_ARGS} > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" 2>&1; rc=$?; echo "prof rc=$rc"
exit $rc
