#!/bin/bash
# Practical fp16 MFMA ceiling (tools/probes/mfma_ceiling.hip) beside the four-wave tiled scan at
# the configs[3] per-rank shape (1.25M rows x 512 queries) and the 1M / G = 8 shape, same box.
TAG=${1:-r02o}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
O=gpurun_out/${TAG}_mfma_ceiling.txt
timeout -k 10 120 ./tools/probes/mfma_ceiling 20000 > $O 2>&1 || exit $?
timeout -k 10 200 python tools/shard_bench.py --chunks 10000000 --gs 8 --k 5 >> $O 2>&1 || exit $?
timeout -k 10 200 python tools/shard_bench.py --chunks 1000000 --gs 8 --k 5 >> $O 2>&1 || exit $?
timeout -k 10 120 ./tools/probes/mfma_ceiling 20000 >> $O 2>&1 || exit $?
grep -v amdgpu.ids $O
