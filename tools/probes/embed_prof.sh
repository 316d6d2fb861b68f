#!/bin/bash
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp; mkdir -p "$R/gpurun_out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${1:-ep}_prof" -o run -- python3 "$R/tools/probes/embed_prof.py" > "$R/gpurun_out/${1:-ep}.log" 2>&1 || exit $?
tail -1 "$R/gpurun_out/${1:-ep}.log"
python3 - "$R/gpurun_out/${1:-ep}_prof/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(r["Name"][:90], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), r["Percentage"][:5])
PY
