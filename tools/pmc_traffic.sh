#!/bin/bash
# PMC traffic of the dominant scan of one bench.py shape: FETCH_SIZE and WRITE_SIZE each in a run
# of its own (no tracing domains), then tools/pmc_traffic.py -> gpurun_out/traffic/<key>.json
# (copied into profiles/traffic/ by hand after review).
# Usage: pmc_traffic.sh TAG FIELD [bench.py args...]   (FIELD: roofline | roofline_sparse)
TAG=$1; FIELD=$2; shift 2
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out/traffic"
B="$R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --latency-iters 2 $*"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/${TAG}_$c" -o run -- python3 $B > "$R/gpurun_out/${TAG}_$c.log" 2>&1 || exit $?
done
F="$R/gpurun_out/${TAG}_FETCH_SIZE/run_counter_collection.csv"
W="$R/gpurun_out/${TAG}_WRITE_SIZE/run_counter_collection.csv"
python3 "$R/tools/pmc_traffic.py" "$F" "$W" "$R/gpurun_out/${TAG}_FETCH_SIZE.log" $FIELD > "$R/gpurun_out/traffic/${TAG}.json" || exit $?
cat "$R/gpurun_out/traffic/${TAG}.json"
