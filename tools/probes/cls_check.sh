#!/bin/bash
# CLS-query attention change check: encoder GPU tests, full-depth rerank parity, rerank bench,
# kernel stats of the rerank bench.
TAG=${1:-r02r}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_encoder_gpu.py tests/test_fullsize_gpu.py -k "encoder or attention or rerank or cross" -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_enc.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/${TAG}_enc.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload hybrid_rerank --steps 5 --warmup 2 --latency-iters 3 --no-cpu-baseline > gpurun_out/${TAG}_bench_rerank.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench_rerank.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("rerank", round(d["value"],1), round(d["ms_per_step"],2), round(d["roofline"]["avg_forward_ms"],2))'
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_rp -o run -- python3 $R/bench.py --workload hybrid_rerank --steps 3 --warmup 1 --latency-iters 1 --no-cpu-baseline > $R/gpurun_out/${TAG}_rp.log 2>&1 || exit $?
python3 $R/tools/rocpd_stats.py $R/gpurun_out/${TAG}_rp/run_results.db > $R/gpurun_out/${TAG}_rerank_kernel_stats.csv || exit $?
rm -rf $R/gpurun_out/${TAG}_rp
grep -E "attention" $R/gpurun_out/${TAG}_rerank_kernel_stats.csv | cut -d, -f1-4
