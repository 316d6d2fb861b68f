#!/bin/bash
# Kernel-trace stats of the sparse top-k chain alone (no concurrent dense scan), 1M rows, 64 queries.
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r01f_prof_sparse" -o run -- \
  python3 "$R/tools/sparse_bench.py" --iters 10 > "$R/gpurun_out/r01f_prof_sparse.log" 2>&1; rc=$?
echo "prof sparse rc=$rc"; exit $rc
