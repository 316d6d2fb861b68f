#!/bin/bash
# Counters of the int8 filter scan (bench.py default): one SQ pass, one TA/TD/GRBM pass.
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
TAG=${1:-pmci8}
B="$R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --latency-iters 2"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD --output-format csv -d "$R/gpurun_out/${TAG}_sq" -o run -- python3 $B > "$R/gpurun_out/${TAG}_sq.log" 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc TA_BUSY_avr TD_BUSY_avr GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$R/gpurun_out/${TAG}_ta" -o run -- python3 $B > "$R/gpurun_out/${TAG}_ta.log" 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d "$R/gpurun_out/${TAG}_l2" -o run -- python3 $B > "$R/gpurun_out/${TAG}_l2.log" 2>&1 || exit $?
for p in sq ta l2; do python3 - "$R/gpurun_out/${TAG}_$p/run_counter_collection.csv" <<'PY' > "$R/gpurun_out/${TAG}_$p.txt"
import csv, collections, sys
acc = collections.defaultdict(lambda: collections.defaultdict(float)); dur = {}
for r in csv.DictReader(open(sys.argv[1])):
    if "scan_i8" not in r["Kernel_Name"] and "dense_scan_kernel" not in r["Kernel_Name"]: continue
    acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for c, d in acc.items():
    print(c, sum(d.values()) / len(d))
print("duration_ns", sum(dur.values()) / max(len(dur), 1))
PY
done
rm -rf "$R/gpurun_out/${TAG}_sq" "$R/gpurun_out/${TAG}_ta" "$R/gpurun_out/${TAG}_l2"
cat "$R/gpurun_out/${TAG}_sq.txt" "$R/gpurun_out/${TAG}_ta.txt" "$R/gpurun_out/${TAG}_l2.txt"
