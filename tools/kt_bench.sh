#!/bin/bash
# kernel-trace summary of one bench configuration: tools/kt_bench.sh TAG <bench args...>
TAG=$1; shift
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}" -o run -- python3 "$R/bench.py" "$@" > "$R/gpurun_out/${TAG}.log" 2>&1
rc=$?; echo "$TAG rc=$rc"; exit $rc
