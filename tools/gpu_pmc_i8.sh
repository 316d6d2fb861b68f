#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes of the 64-query int8 scan (the first pass only: the collect
# pass instantiation <.., false, true> shares the name prefix and reads ~nothing).
TAG=${1:-pmc}
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --latency-iters 2"
P="$R/gpurun_out/${TAG}_p"; mkdir -p "$P"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$P/fetch" -o run -- python3 $B > "$P/fetch.log" 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$P/write" -o run -- python3 $B > "$P/write.log" 2>&1 || exit $?
python3 "$R/tools/pmc_traffic.py" "$P/fetch/run_counter_collection.csv" "$P/write/run_counter_collection.csv" "dense_scan_i8_kernel<1024, false, false>" 1032131072 "bench.py default: 1M x 1024 rows, int8 filter image (tile-blocked, scattered row order) + a32/e32, 64 fp16 queries per launch" > "$R/gpurun_out/${TAG}_dense_scan_i8_traffic.json" || exit $?
rm -rf "$P"
cat "$R/gpurun_out/${TAG}_dense_scan_i8_traffic.json"
