#!/bin/bash
# Dense parity, then per-GPU compute of the sharded step (G = 4, 8 at 1M; G = 8 at 10M, both stagings).
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dense_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gq_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gq_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/shard_bench.py --gs 4,8 > gpurun_out/gq_sb.log 2>&1 || exit $?
tail -2 gpurun_out/gq_sb.log
for st in glds reg glds; do
  ARMI_GEMM_STAGE=$st timeout -k 10 300 python tools/shard_bench.py --gs 8 --chunks 10000000 --iters 10 > gpurun_out/gq_sb10m_$st.log 2>&1 || exit $?
  echo "10M stage=$st $(tail -1 gpurun_out/gq_sb10m_$st.log)"
done
