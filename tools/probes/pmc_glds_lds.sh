#!/bin/bash
# SQ counters of the branch-free LDS-DMA tiled scan at the 10M / 8-way per-rank shape (one
# pass, 8 SQ counters): MFMA busy, LDS activity and bank conflicts.
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
B="$R/tools/shard_bench.py --gs 8 --chunks 10000000 --iters 5"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_INST_LDS --output-format csv -d "$R/gpurun_out/pmcl_sq" -o run -- python3 $B > "$R/gpurun_out/pmcl_sq.log" 2>&1; rc=$?; echo "sq rc=$rc"
exit $rc
