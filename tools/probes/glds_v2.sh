#!/bin/bash
# Branch-free LDS-DMA tiled scan: dense GPU parity tests, then per-rank scan time at the
# 1M G=1..8 and 10M/8-way shapes, plus the register-staged form on the same box for A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dense_gpu.py tests/test_store_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v2_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc: $(tail -1 gpurun_out/v2_pytest.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/shard_bench.py > gpurun_out/v2_shard.log 2>&1 || exit $?
timeout -k 10 200 python tools/shard_bench.py --chunks 10000000 --gs 8 --k 5 >> gpurun_out/v2_shard.log 2>&1 || exit $?
timeout -k 10 200 python tools/shard_bench.py --chunks 10000000 --gs 8 --k 40 >> gpurun_out/v2_shard.log 2>&1 || exit $?
ARMI_GEMM_STAGE=reg timeout -k 10 200 python tools/shard_bench.py --chunks 10000000 --gs 8 --k 5 >> gpurun_out/v2_shard.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/v2_shard.log
