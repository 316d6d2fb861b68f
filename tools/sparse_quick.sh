#!/bin/bash
# sparse parity tests + micro-benchmark variants + kernel trace of the micro-benchmark
TAG=${1:-sq}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_sparse_rrf_gpu.py tests/test_golden_pipeline_gpu.py -q -m "gpu and not slow" > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for d in ${DBGS:-0}; do
  ARMI_SPARSE_DBG=$d timeout -k 10 300 python tools/sparse_bench.py > gpurun_out/${TAG}_dbg$d.log 2>&1 || exit $?
  echo "dbg=$d $(tail -1 gpurun_out/${TAG}_dbg$d.log)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_kt" -o run -- python3 "$GRAFT_REPO_ROOT/tools/sparse_bench.py" > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_kt.log" 2>&1; rc=$?; echo "kt rc=$rc"
exit $rc
