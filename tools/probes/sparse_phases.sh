#!/bin/bash
# Phase timers of sparse_scan_kernel (profiling build, ARMI_SPARSE_PROFILE) in the hybrid bench,
# plus the ARMI_SPARSE_DBG ablations (1 = no compute, 2 = stage nothing, 4 = no step barrier).
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
L=audio_rag_amd/_lib
cp $L/libarmi.so $L/libarmi_norm.so && cp $L/libarmi_prof.so $L/libarmi.so
for d in 8 9 10 12 14; do
  ARMI_SPARSE_DBG=$d timeout -k 10 200 python bench.py --workload hybrid --steps 10 --warmup 2 --no-cpu-baseline \
    > gpurun_out/sph_$d.log 2>&1 || { cp $L/libarmi_norm.so $L/libarmi.so; exit 1; }
  echo "dbg=$d: $(grep 'sparse prof' gpurun_out/sph_$d.log | tail -1)"
  python -c "import json;d=json.loads(open('gpurun_out/sph_$d.log').read().strip().splitlines()[-1]);print('   step ms', round(d['ms_per_step'],4))"
done
cp $L/libarmi_norm.so $L/libarmi.so
