#!/bin/bash
# Tiled scan at the 10M / 8-way per-rank shape with rows streamed from HBM (0) vs re-read from
# L2 (ARMI_GEMM_ABLATE=8: every step reads the range's first row tile; results invalid).
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
for a in 0 8 0 8; do
  ARMI_GEMM_ABLATE=$a timeout -k 10 200 python tools/shard_bench.py --gs 8 --chunks 10000000 --iters 10 > gpurun_out/ablate_$a.log 2>&1 || exit $?
  echo "ablate=$a $(tail -1 gpurun_out/ablate_$a.log)"
done
