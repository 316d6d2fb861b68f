#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for d in 0 1 2 4 3 7; do
  ARMI_SPARSE_DBG=$d timeout -k 10 300 python tools/sparse_bench.py "$@" > gpurun_out/sdbg_$d.log 2>&1 || exit $?
  echo "dbg=$d $(tail -1 gpurun_out/sdbg_$d.log)"
done
