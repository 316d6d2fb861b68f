#!/bin/bash
# PMC passes over the sparse micro-benchmark (one counter group per pass)
TAG=${1:-spb}
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/${TAG}_p$i" -o run -- python3 "$R/tools/sparse_bench.py" --iters 4 > "$R/gpurun_out/${TAG}_p$i.log" 2>&1; rc=$?
  echo "pass $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done <<GROUPS
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES
SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_ANY
SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD
GROUPS
