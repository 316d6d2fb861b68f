#!/bin/bash
# dense_merge_kernel phase costs (probe builds, results wrong): ARMI_MERGE_ABL=3 loads + query
# norm only, 2 up to the sorted selection, 1 rescore loads all from one (cached) row; kernel
# average from a kernel trace of the dense bench for each build.
TAG=${1:-mph}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
export TMPDIR=/tmp
for a in 0 3 2 1; do
  if [ $a != 0 ]; then
    ARMI_BUILD_FLAGS="-DARMI_PROBE_BUILD -DARMI_MERGE_ABL=$a" timeout -k 10 300 python -c "from audio_rag_amd import build; build.build()" > gpurun_out/${TAG}_build$a.log 2>&1 || exit $?
  fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/${TAG}_$a -o run -- python3 $R/bench.py --steps 100 --warmup 5 --no-cpu-baseline --latency-iters 2 > gpurun_out/${TAG}_$a.log 2>&1 || exit $?
  python3 $R/tools/rocpd_stats.py /tmp/${TAG}_$a/run_results.db > gpurun_out/${TAG}_stats_$a.csv || exit $?
  echo "abl=$a merge: $(grep dense_merge_kernel gpurun_out/${TAG}_stats_$a.csv | cut -d, -f4) ns"
done
