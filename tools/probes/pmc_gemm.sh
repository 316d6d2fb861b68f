#!/bin/bash
# SQ counters of the LDS-DMA tiled scan at the 10M / 8-way per-rank shape (one pass, 8 SQ
# counters) plus a TA/TD pass.
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
B="$R/tools/shard_bench.py --gs 8 --chunks 10000000 --iters 5"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d "$R/gpurun_out/pmcg_sq" -o run -- python3 $B > "$R/gpurun_out/pmcg_sq.log" 2>&1; rc=$?; echo "sq rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TD_BUSY_avr --output-format csv -d "$R/gpurun_out/pmcg_ta" -o run -- python3 $B > "$R/gpurun_out/pmcg_ta.log" 2>&1; rc=$?; echo "ta rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d "$R/gpurun_out/pmcg_l2" -o run -- python3 $B > "$R/gpurun_out/pmcg_l2.log" 2>&1; rc=$?; echo "l2 rc=$rc"
exit $rc
