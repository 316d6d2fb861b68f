#!/bin/bash
# Ablations of the LDS-DMA tiled scan at the 10M / 8-way per-rank shape (scan-kernel time only).
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
for a in 0 16 32 64 80 48 112; do
  ARMI_GEMM_ABLATE=$a timeout -k 10 200 python tools/shard_bench.py --gs 8 --chunks 10000000 --iters 3 > gpurun_out/abl_$a.log 2>&1 || exit $?
  echo "ablate=$a $(tail -1 gpurun_out/abl_$a.log | sed "s/.*scan kernel/scan kernel/")"
done
