#!/bin/bash
TAG=${1:-sp}
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
B="$R/bench.py --workload hybrid --steps 6 --warmup 1 --latency-iters 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_kt" -o run -- python3 $B > "$R/gpurun_out/${TAG}_kt.log" 2>&1; rc=$?; echo "kt rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$R/gpurun_out/${TAG}_sq" -o run -- python3 $B > "$R/gpurun_out/${TAG}_sq.log" 2>&1; rc=$?; echo "sq rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_RD TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$R/gpurun_out/${TAG}_sq2" -o run -- python3 $B > "$R/gpurun_out/${TAG}_sq2.log" 2>&1; rc=$?; echo "sq2 rc=$rc"
exit 0
