#!/bin/bash
# Phase timers of sparse_scan_kernel (profiling build ablibs/libarmi_sprof.so, ARMI_SPARSE_PROFILE,
# loaded through ARMI_LIB_PATH) in the hybrid bench, plus the ARMI_SPARSE_DBG ablations
# (1 = no compute, 2 = stage nothing, 4 = no step barrier; 8 = report).
TAG=${1:-sph}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
for d in ${DBGS:-8 9 10 11 12 15}; do
  ARMI_LIB_PATH=ablibs/libarmi_sprof.so ARMI_SPARSE_DBG=$d timeout -k 10 200 python bench.py --workload hybrid --eager-hybrid --steps 10 --warmup 2 --no-cpu-baseline --no-extras \
    > gpurun_out/${TAG}_$d.log 2>&1 || exit 1
  # the first report is a 64-query pass (the bench's single-query latency calls come last)
  echo "dbg=$d: $(grep 'sparse prof' gpurun_out/${TAG}_$d.log | head -1)"
  python -c "import json;d=json.loads(open('gpurun_out/${TAG}_$d.log').read().strip().splitlines()[-1]);print('   step ms', round(d['ms_per_step'],4), 'sparse scan ms', round(d['roofline_sparse']['avg_launch_ms'],4))"
done
