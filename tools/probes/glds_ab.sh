#!/bin/bash
# Parity of the LDS-DMA tiled scan (default ARMI_GEMM_STAGE=glds) on the dense GPU tests, then
# per-GPU compute of the sharded step with register vs LDS-DMA staging (G = 4, 8 at 1M chunks;
# G = 8 at 10M).
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dense_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/glds_tests.log 2>&1; rc=$?
tail -3 gpurun_out/glds_tests.log
[ $rc -eq 0 ] || exit $rc
for st in reg glds reg glds; do
  ARMI_GEMM_STAGE=$st timeout -k 10 200 python tools/shard_bench.py --gs 4,8 > gpurun_out/glds_sb_$st.log 2>&1 || exit $?
  echo "stage=$st"; tail -2 gpurun_out/glds_sb_$st.log
done
for st in reg glds; do
  ARMI_GEMM_STAGE=$st timeout -k 10 300 python tools/shard_bench.py --gs 8 --chunks 10000000 > gpurun_out/glds_sb10m_$st.log 2>&1 || exit $?
  echo "10M stage=$st $(tail -1 gpurun_out/glds_sb10m_$st.log)"
done
