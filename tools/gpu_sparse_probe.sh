#!/bin/bash
# Sparse stage alone at 1M rows: filter on / off timings, then a kernel trace of the filter run.
TAG=${1:-sp}
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 1
for f in on off; do
  timeout -k 10 200 python tools/sparse_bench.py --k ${K:-40} --iters 50 --filter $f >> gpurun_out/${TAG}_sparse.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}" -o run -- python3 "$R/tools/sparse_bench.py" --k ${K:-40} --iters 50 --filter on > "$R/gpurun_out/${TAG}_sparse_prof.log" 2>&1; rc=$?; echo "prof rc=$rc"
exit $rc
