#!/bin/bash
# Ablations of the phase-pipelined tiled scan (probe build, results wrong) at the 10M / 8-way
# per-rank shape: which part of the phase (DMA wait, HBM rows, MFMAs, barriers) costs the time.
TAG=${1:-p8abl}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
ARMI_BUILD_FLAGS=-DARMI_PROBE_BUILD timeout -k 10 300 python -c "from audio_rag_amd import build; build.build()" > gpurun_out/${TAG}_build.log 2>&1 || exit $?
for a in ${ABLS:-0 1 2 3 4 8 12 13 0}; do
  ARMI_GEMM_ABLATE=$a timeout -k 10 200 python tools/shard_bench.py --chunks 10000000 --gs 8 --iters 10 > gpurun_out/${TAG}_$a.log 2>&1 || exit $?
  echo "ablate=$a $(grep -o 'scan kernel.*' gpurun_out/${TAG}_$a.log)"
done
