#!/bin/bash
# full GPU check: all non-slow GPU tests, sparse micro-bench (+ phase profile), dense + hybrid bench
TAG=${1:-gr}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m "gpu and not slow" > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for d in ${DBGS:-0 8}; do
  ARMI_SPARSE_DBG=$d timeout -k 10 300 python tools/sparse_bench.py > gpurun_out/${TAG}_dbg$d.log 2>&1 || exit $?
  echo "dbg=$d $(grep -h 'prof\|batch' gpurun_out/${TAG}_dbg$d.log | tail -2 | tr '\n' ' ')"
done
for w in dense hybrid; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 > gpurun_out/${TAG}_bench_$w.log 2>&1 || exit $?
  echo "$w $(tail -1 gpurun_out/${TAG}_bench_$w.log | cut -c1-330)"
done
