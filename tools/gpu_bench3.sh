#!/bin/bash
# The three bench lines that carry a cpu_baseline (dense headline, hybrid, hybrid_rerank).
TAG=${1:-b3}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench_dense.log 2>&1 || exit $?
echo "dense: $(tail -1 gpurun_out/${TAG}_bench_dense.log | cut -c1-200)"
timeout -k 10 400 python bench.py --workload hybrid --steps 20 --warmup 3 > gpurun_out/${TAG}_bench_hybrid.log 2>&1 || exit $?
echo "hybrid: $(tail -1 gpurun_out/${TAG}_bench_hybrid.log | cut -c1-200)"
timeout -k 10 500 python bench.py --workload hybrid_rerank --steps 5 --warmup 2 --latency-iters 3 \
  > gpurun_out/${TAG}_bench_rerank.log 2>&1 || exit $?
echo "rerank: $(tail -1 gpurun_out/${TAG}_bench_rerank.log | cut -c1-200)"
