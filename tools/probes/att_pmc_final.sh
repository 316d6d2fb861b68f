#!/bin/bash
# SQ / GRBM / FETCH counters of the product attention_f16_kernel at the configs[2] shape.
TAG=${1:-attpmc}
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
P="$R/tools/probes/att_one.py"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d "$R/gpurun_out/${TAG}_sq" -o run -- python3 $P > "$R/gpurun_out/${TAG}_sq.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVES SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$R/gpurun_out/${TAG}_sq2" -o run -- python3 $P > "$R/gpurun_out/${TAG}_sq2.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/${TAG}_fetch" -o run -- python3 $P > "$R/gpurun_out/${TAG}_fetch.log" 2>&1 || exit $?
cd "$R"
python3 tools/pmc_summary.py attention_f16_kernel gpurun_out/${TAG}_sq/run_counter_collection.csv gpurun_out/${TAG}_sq2/run_counter_collection.csv gpurun_out/${TAG}_fetch/run_counter_collection.csv > gpurun_out/${TAG}_summary.txt
rm -rf gpurun_out/${TAG}_sq gpurun_out/${TAG}_sq2 gpurun_out/${TAG}_fetch
cat gpurun_out/${TAG}_summary.txt
