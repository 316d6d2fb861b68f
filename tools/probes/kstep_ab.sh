#!/bin/bash
# Dense parity with k-step 32 (default) and 64, then the 10M / 8-way per-rank scan with both.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
for ks in 32 64; do
  ARMI_GEMM_KSTEP=$ks timeout -k 10 400 python -u -m pytest tests/test_dense_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ks_tests_$ks.log 2>&1; rc=$?
  echo "ks=$ks $(tail -1 gpurun_out/ks_tests_$ks.log)"
  [ $rc -eq 0 ] || exit $rc
done
for ks in 32 64 32 64; do
  ARMI_GEMM_KSTEP=$ks timeout -k 10 300 python tools/shard_bench.py --gs 4,8 > gpurun_out/ks_sb_$ks.log 2>&1 || exit $?
  ARMI_GEMM_KSTEP=$ks timeout -k 10 300 python tools/shard_bench.py --gs 8 --chunks 10000000 --iters 10 > gpurun_out/ks_sb10m_$ks.log 2>&1 || exit $?
  echo "ks=$ks"; tail -2 gpurun_out/ks_sb_$ks.log; tail -1 gpurun_out/ks_sb10m_$ks.log
done
