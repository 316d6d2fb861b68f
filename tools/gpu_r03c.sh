#!/bin/bash
# Round-3: GEMM parity + speed vs hipBLASLt, dense collect tests after the ordinal-list change,
# and the int8-scan phase stamps.
TAG=${1:-r03c}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gemm_gpu.py tests/test_dense_collect_gpu.py tests/test_dense_filter_gpu.py \
  > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/probes/gemm_bench.py > gpurun_out/${TAG}_gemm.log 2>&1 || exit $?
cat gpurun_out/${TAG}_gemm.log
ARMI_GEMM_BARRIERS=2 timeout -k 10 300 python tools/probes/gemm_bench.py > gpurun_out/${TAG}_gemm_b2.log 2>&1 || exit $?
echo "barriers=2:"; cat gpurun_out/${TAG}_gemm_b2.log
bash tools/probes/i8_stamps.sh ${TAG}stp
