#!/bin/bash
# Sparse scan alone (tools/sparse_bench.py, 1M rows, 64-query batches): time, rocprofv3 kernel
# stats, then the profiling build's phase timers with the ARMI_SPARSE_DBG ablations
# (8 = report, 9 = no compute, 10 = stage nothing, 12 = no step barrier).
TAG=${1:-iso}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
export TMPDIR=/tmp
L=audio_rag_amd/_lib
timeout -k 10 300 python tools/sparse_bench.py --iters 50 > gpurun_out/${TAG}_sb.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_sb.log
P=/tmp/${TAG}_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P -o run -- python3 tools/sparse_bench.py --iters 50 > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python3 tools/rocpd_stats.py $P/run_results.db > gpurun_out/${TAG}_kernel_stats.csv || exit 1
cut -c1-150 gpurun_out/${TAG}_kernel_stats.csv | head -10
[ -f $L/libarmi_prof.so ] || exit 0
cp $L/libarmi.so $L/libarmi_norm.so && cp $L/libarmi_prof.so $L/libarmi.so
for d in 8 9 10 12; do
  ARMI_SPARSE_DBG=$d timeout -k 10 200 python tools/sparse_bench.py --iters 5 > gpurun_out/${TAG}_sph_$d.log 2>&1 || { cp $L/libarmi_norm.so $L/libarmi.so; exit 1; }
  echo "dbg=$d: $(grep 'sparse prof' gpurun_out/${TAG}_sph_$d.log | tail -1 | cut -c40-)"
  echo "   $(tail -1 gpurun_out/${TAG}_sph_$d.log)"
done
cp $L/libarmi_norm.so $L/libarmi.so
