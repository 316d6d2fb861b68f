#!/bin/bash
# Phase timers (ARMI_SPARSE_DBG=8) of sparse_scan_kernel for several probe builds in the eager
# hybrid bench: tools/probes/sparse_variants.sh TAG lib1 lib2 ...
TAG=$1; shift
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
for lib in "$@"; do
  n=$(basename $lib .so)
  ARMI_LIB_PATH=$lib ARMI_SPARSE_DBG=8 timeout -k 10 200 python bench.py --workload hybrid --eager-hybrid --steps 10 --warmup 2 --no-cpu-baseline --no-extras \
    > gpurun_out/${TAG}_$n.log 2>&1 || exit 1
  echo "$n: $(grep 'sparse prof' gpurun_out/${TAG}_$n.log | head -1)"
  python -c "import json;d=json.loads(open('gpurun_out/${TAG}_$n.log').read().strip().splitlines()[-1]);print('   step ms', round(d['ms_per_step'],4), 'sparse scan ms', round(d['roofline_sparse']['avg_launch_ms'],4))"
done
