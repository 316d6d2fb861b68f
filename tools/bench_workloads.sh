#!/bin/bash
# Runs the non-default bench workloads (each step under its own limit).
TAG=${1:-wl}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload hybrid --steps 20 --warmup 3 > gpurun_out/${TAG}_hybrid.log 2>&1; rc=$?; echo "hybrid rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload hybrid_rerank --rerank-dtype bf16 --steps 5 --warmup 1 --latency-iters 3 > gpurun_out/${TAG}_rerank_bf16.log 2>&1; rc=$?; echo "rerank bf16 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload hybrid_rerank --rerank-dtype fp32 --steps 3 --warmup 1 --latency-iters 2 > gpurun_out/${TAG}_rerank_fp32.log 2>&1; rc=$?; echo "rerank fp32 rc=$rc"
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_hybrid" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload hybrid --steps 10 --warmup 2 --latency-iters 2 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_hybrid.log" 2>&1; rc=$?; echo "prof rc=$rc"
exit $rc
