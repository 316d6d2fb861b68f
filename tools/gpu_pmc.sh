#!/bin/bash
# Two PMC passes (instruction mix, wait and MFMA-busy cycles) over one command, one rocprofv3 run
# per counter set; summary of kernels whose name contains $PMC_MATCH. Usage: gpu_pmc.sh TAG CMD...
TAG=$1; shift
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $set --output-format csv -d "$R/gpurun_out/${TAG}_p$i" -o run -- "$@" > "$R/gpurun_out/${TAG}_p$i.log" 2>&1 || exit $?
done
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/${TAG}_p1/run_counter_collection.csv" "$R/gpurun_out/${TAG}_p2/run_counter_collection.csv" > "$R/gpurun_out/${TAG}_summary.txt"
cat "$R/gpurun_out/${TAG}_summary.txt"
