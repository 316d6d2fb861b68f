#!/bin/bash
# SQ / GRBM counters of linear_f16_kernel on one cross-encoder GEMM shape (tools/probes/gemm_bench.py,
# GEMM_SHAPES=<shape>, hipBLASLt arm skipped): two SQ passes + a GRBM pass (effective clock).
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
TAG=${1:-pmclin}
export GEMM_SHAPES=${2:-qkv} GEMM_NO_LT=1
B="$R/tools/probes/gemm_bench.py"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d "$R/gpurun_out/${TAG}_a" -o run -- python3 $B > "$R/gpurun_out/${TAG}_a.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_MFMA --output-format csv -d "$R/gpurun_out/${TAG}_b" -o run -- python3 $B > "$R/gpurun_out/${TAG}_b.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$R/gpurun_out/${TAG}_c" -o run -- python3 $B > "$R/gpurun_out/${TAG}_c.log" 2>&1 || exit $?
for p in a b c; do python3 - "$R/gpurun_out/${TAG}_$p/run_counter_collection.csv" <<'PY' > "$R/gpurun_out/${TAG}_$p.txt"
import csv, collections, sys
acc = collections.defaultdict(lambda: collections.defaultdict(float)); dur = {}
for r in csv.DictReader(open(sys.argv[1])):
    if "linear_f16_kernel" not in r["Kernel_Name"]: continue
    acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for c, d in sorted(acc.items()):
    print(c, sum(d.values()) / len(d))
print("duration_ns", sum(dur.values()) / max(len(dur), 1))
PY
done
rm -rf "$R/gpurun_out/${TAG}_a" "$R/gpurun_out/${TAG}_b" "$R/gpurun_out/${TAG}_c"
cat "$R/gpurun_out/${TAG}_a.txt" "$R/gpurun_out/${TAG}_b.txt" "$R/gpurun_out/${TAG}_c.txt"
