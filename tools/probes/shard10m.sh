#!/bin/bash
# Per-rank compute of configs[3] (10M chunks sharded 8-way: 1.25M rows x 512 queries) with the
# default LDS-DMA tiled scan and, for A/B, the register-staged form. Each step has its own limit.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/shard10m.log
timeout -k 10 200 python tools/shard_bench.py --chunks 10000000 --gs 8 --k 5 > $O 2>&1 || exit $?
timeout -k 10 200 python tools/shard_bench.py --chunks 10000000 --gs 8 --k 40 >> $O 2>&1 || exit $?
ARMI_GEMM_STAGE=reg timeout -k 10 200 python tools/shard_bench.py --chunks 10000000 --gs 8 --k 5 >> $O 2>&1 || exit $?
grep -v amdgpu.ids $O
