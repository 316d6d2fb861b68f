#!/bin/bash
# Counters of the tiled scan at the 10M / 8-way per-rank shape for both schedules (p8, glds):
# one SQ pass, one TA/TD/GRBM pass, one L2 pass per form; each pass its own run.
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
TAG=${1:-pmcp8}
B="$R/tools/shard_bench.py --gs 8 --chunks 10000000 --iters 5"
for f in p8 glds; do
  export ARMI_GEMM_FORM=$f
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d "$R/gpurun_out/${TAG}_${f}_sq" -o run -- python3 $B > "$R/gpurun_out/${TAG}_${f}_sq.log" 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TD_BUSY_avr GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$R/gpurun_out/${TAG}_${f}_ta" -o run -- python3 $B > "$R/gpurun_out/${TAG}_${f}_ta.log" 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$R/gpurun_out/${TAG}_${f}_l2" -o run -- python3 $B > "$R/gpurun_out/${TAG}_${f}_l2.log" 2>&1 || exit $?
  echo "$f done"
done
