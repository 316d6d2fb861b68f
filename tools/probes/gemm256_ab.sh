#!/bin/bash
# Parity of the 256-row tiled scan (ARMI_GEMM_ROWS=256) on the dense GPU tests, then per-GPU
# compute of the sharded step with both row tiles (G = 4, 8 at 1M chunks; G = 8 at 10M).
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
ARMI_GEMM_ROWS=256 timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/g256_tests.log 2>&1; rc=$?
tail -3 gpurun_out/g256_tests.log
[ $rc -eq 0 ] || exit $rc
for rows in 128 256 128 256; do
  ARMI_GEMM_ROWS=$rows timeout -k 10 200 python tools/shard_bench.py --gs 4,8 > gpurun_out/g256_sb_$rows.log 2>&1 || exit $?
  echo "rows=$rows"; tail -3 gpurun_out/g256_sb_$rows.log
done
for rows in 128 256; do
  ARMI_GEMM_ROWS=$rows timeout -k 10 300 python tools/shard_bench.py --gs 8 --chunks 10000000 > gpurun_out/g256_sb10m_$rows.log 2>&1 || exit $?
  echo "10M rows=$rows"; tail -2 gpurun_out/g256_sb10m_$rows.log
done
