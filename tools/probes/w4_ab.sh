#!/bin/bash
# Four-wave tiled scan (w4) vs the four-stage LDS-DMA scan (glds): parity tests of the
# tiled path, then per-rank scan time at the G = 4 / 8 shapes of 1M rows and at 10M / 8.
TAG=${1:-w4}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
ARMI_GEMM_FORM=w4 timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py tests/test_fullsize_gpu.py -k "not bge and not rerank and not hybrid" \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
for f in w4 glds w4; do
  ARMI_GEMM_FORM=$f timeout -k 10 200 python tools/shard_bench.py --gs 4,8 > gpurun_out/${TAG}_$f.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/${TAG}_$f.log | sed "s/^/$f: /"
  ARMI_GEMM_FORM=$f timeout -k 10 300 python tools/shard_bench.py --chunks 10000000 --gs 8 > gpurun_out/${TAG}_${f}_10m.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/${TAG}_${f}_10m.log | sed "s/^/$f 10M: /"
done
