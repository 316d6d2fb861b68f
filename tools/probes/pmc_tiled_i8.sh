#!/bin/bash
# Counters of the int8 tiled scan (dense_gemm_scan_w4_kernel<1024, 0, true>) at the configs[3]
# per-rank shape (1.25M rows x 512 queries, top-5; tools/shard_bench.py --gs 8 --chunks 10M):
# an SQ pass, a second SQ pass, GRBM (clock), FETCH_SIZE and WRITE_SIZE passes.
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
TAG=${1:-pmcti8}
B="$R/tools/shard_bench.py --gs 8 --chunks 10000000 --iters 5"
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/${TAG}_$name" -o run -- python3 $B > "$R/gpurun_out/${TAG}_$name.log" 2>&1 || exit $?
}
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS
run b SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
run c GRBM_GUI_ACTIVE GRBM_COUNT
run f FETCH_SIZE
run w WRITE_SIZE
for p in a b c f w; do python3 - "$R/gpurun_out/${TAG}_$p/run_counter_collection.csv" <<'PY' > "$R/gpurun_out/${TAG}_$p.txt"
import csv, collections, sys
acc = collections.defaultdict(lambda: collections.defaultdict(float)); dur = {}
for r in csv.DictReader(open(sys.argv[1])):
    if "dense_gemm_scan_w4_kernel" not in r["Kernel_Name"]: continue
    acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for c, d in sorted(acc.items()):
    print(c, sum(d.values()) / len(d))
print("duration_ns", sum(dur.values()) / max(len(dur), 1))
PY
done
rm -rf "$R/gpurun_out/${TAG}_"{a,b,c,f,w}
cat "$R/gpurun_out/${TAG}_"{a,b,c,f,w}.txt
