#!/bin/bash
# One GPU session: full -m gpu suite, the three bench workloads, a kernel-trace profile of the
# default bench. Every GPU step has its own time limit; a crash / timeout ends the session.
TAG=${1:-full}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc: $(tail -1 gpurun_out/${TAG}_pytest.log)"
ok $rc || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench_dense.log 2>&1 || exit $?
echo "dense: $(tail -1 gpurun_out/${TAG}_bench_dense.log | cut -c1-400)"
timeout -k 10 300 python bench.py --workload hybrid --steps 20 --warmup 3 \
  > gpurun_out/${TAG}_bench_hybrid.log 2>&1 || exit $?
echo "hybrid: $(tail -1 gpurun_out/${TAG}_bench_hybrid.log | cut -c1-300)"
timeout -k 10 400 python bench.py --workload hybrid_rerank --steps 5 --warmup 2 --latency-iters 3 \
  > gpurun_out/${TAG}_bench_rerank.log 2>&1 || exit $?
echo "rerank: $(tail -1 gpurun_out/${TAG}_bench_rerank.log | cut -c1-300)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_dense" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --latency-iters 3 \
  > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_dense.log" 2>&1; rc=$?
echo "prof dense rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_rerank" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --workload hybrid_rerank --steps 3 --warmup 1 --latency-iters 1 \
  > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_rerank.log" 2>&1; rc=$?
echo "prof rerank rc=$rc"
exit $rc
