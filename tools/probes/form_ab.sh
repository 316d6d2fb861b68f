#!/bin/bash
# Scan-form A/B at the G = 2 and G = 4 per-rank shapes (1M rows / G, G*64 queries):
# XCD-grouped 64-query scan vs the LDS-DMA tiled scan.
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
for f in grouped tiled; do
  ARMI_DENSE_SCAN=$f timeout -k 10 200 python tools/shard_bench.py --gs 2,4 > gpurun_out/form_$f.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/form_$f.log | sed "s/^/$f: /"
done
