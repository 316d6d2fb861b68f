#!/bin/bash
# Dense merge change check: dense parity tests, the headline bench, and the merge kernel's
# average duration from a kernel trace of the bench.
TAG=${1:-r02l}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py tests/test_dense_filter_gpu.py tests/test_shards_gpu.py tests/test_store_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_dense_tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/${TAG}_dense_tests.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench_dense.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench_dense.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("dense", round(d["value"]), round(d["ms_per_step"],4), round(d["p50_ms"],4), round(d["roofline"]["avg_launch_ms"],4))'
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_mp -o run -- python3 $R/bench.py --steps 100 --warmup 5 --no-cpu-baseline --latency-iters 2 > $R/gpurun_out/${TAG}_mp.log 2>&1 || exit $?
python3 $R/tools/rocpd_stats.py $R/gpurun_out/${TAG}_mp/run_results.db > $R/gpurun_out/${TAG}_dense_kernel_stats.csv || exit $?
rm -rf $R/gpurun_out/${TAG}_mp
grep -E "merge|scan_i8|exact" $R/gpurun_out/${TAG}_dense_kernel_stats.csv | cut -d, -f1-4 | cut -c1-40,100-200
