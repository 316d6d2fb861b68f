#!/bin/bash
# Four-wave tiled scan: parity (ARMI_GEMM_FORM=w4), w4 vs glds at the 10M / 8-way per-rank shape,
# then ablations of w4 in a probe build (results wrong): 1 no LDS-DMA pieces, 2 no epilogue,
# 3 neither, 4 no MFMAs, 8 no mid-step barrier, 9 no pieces and no barrier.
TAG=${1:-w4x}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
ARMI_GEMM_FORM=w4 timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py tests/test_fullsize_gpu.py -k "not bge and not rerank and not hybrid" \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
for f in w4 glds; do
  ARMI_GEMM_FORM=$f timeout -k 10 300 python tools/shard_bench.py --chunks 10000000 --gs 8 > gpurun_out/${TAG}_${f}_10m.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/${TAG}_${f}_10m.log | sed "s/^/$f 10M: /"
done
ARMI_BUILD_FLAGS=-DARMI_PROBE_BUILD timeout -k 10 300 python -c "from audio_rag_amd import build; build.build()" > gpurun_out/${TAG}_build.log 2>&1 || exit $?
for a in 1 2 3 4 8 9; do
  ARMI_GEMM_FORM=w4 ARMI_GEMM_ABLATE=$a timeout -k 10 300 python tools/shard_bench.py --chunks 10000000 --gs 8 > gpurun_out/${TAG}_abl$a.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/${TAG}_abl$a.log | sed "s/^/w4 ablate $a: /"
done
