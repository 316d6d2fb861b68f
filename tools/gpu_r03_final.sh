#!/bin/bash
# Round-3 measurement session: full -m gpu suite, smoke, every bench workload (dense / hybrid /
# hybrid_rerank with cpu_baseline; stream dense + hybrid; pipeline), rocprofv3 kernel stats of
# the dense and rerank benches, FETCH_SIZE / WRITE_SIZE passes of the dense scan.
TAG=${1:-r03f}
PART=${2:-A}   # A: tests, smoke, dense / hybrid / rerank benches; B: stream, pipeline, profiles
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
j() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($2)"; }
if [ "$PART" = A ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
echo "smoke ok"
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench_dense.log 2>&1 || exit $?
echo "dense: $(j gpurun_out/${TAG}_bench_dense.log 'round(d["value"]), round(d["ms_per_step"],3), round(d["p50_ms"],3), d["roofline"]["kernel"], round(d["roofline"]["frac"],3), d["roofline"]["traffic"], round(d["cpu_baseline"]["value"],1)')"
echo "configs1: $(j gpurun_out/${TAG}_bench_dense.log 'round(d["configs1"]["value"]), round(d["configs1"]["ms_per_step"],4)')"
echo "configs2: $(j gpurun_out/${TAG}_bench_dense.log 'round(d["configs2"]["value"],1), round(d["configs2"]["ms_per_step"],2), round(d["configs2"]["roofline_scan"]["avg_launch_ms"],4)')"
timeout -k 10 300 python bench.py --corpus clustered --no-extras --no-cpu-baseline > gpurun_out/${TAG}_bench_clustered.log 2>&1 || exit $?
echo "clustered: $(j gpurun_out/${TAG}_bench_clustered.log 'round(d["value"]), round(d["ms_per_step"],4), d["certified_frac"]')"
timeout -k 10 600 python bench.py --workload hybrid > gpurun_out/${TAG}_bench_hybrid.log 2>&1 || exit $?
echo "hybrid: $(j gpurun_out/${TAG}_bench_hybrid.log 'round(d["value"]), round(d["ms_per_step"],3), round(d["cpu_baseline"]["value"],2)')"
timeout -k 10 700 python bench.py --workload hybrid_rerank --steps 5 --warmup 2 --latency-iters 3 > gpurun_out/${TAG}_bench_rerank.log 2>&1 || exit $?
echo "rerank: $(j gpurun_out/${TAG}_bench_rerank.log 'round(d["value"],1), round(d["ms_per_step"],2), round(d["roofline"]["avg_forward_ms"],2), round(d["roofline"]["frac"],3), round(d["roofline_scan"]["avg_launch_ms"],4), round(d["cpu_baseline"]["value"],3)')"
RR="--workload hybrid_rerank --steps 4 --warmup 2 --latency-iters 1 --no-cpu-baseline"
ARMI_ATTENTION=persist timeout -k 10 400 python bench.py $RR > gpurun_out/${TAG}_rerank_persist.log 2>&1 || exit $?
echo "rerank persistent attention: $(j gpurun_out/${TAG}_rerank_persist.log 'round(d["value"],1), round(d["roofline"]["avg_forward_ms"],2)')"
ARMI_RERANK_GEMM=torch timeout -k 10 400 python bench.py $RR > gpurun_out/${TAG}_rerank_torchgemm.log 2>&1 || exit $?
echo "rerank hipBLASLt + GELU pass: $(j gpurun_out/${TAG}_rerank_torchgemm.log 'round(d["value"],1), round(d["roofline"]["avg_forward_ms"],2)')"
exit 0
fi
for q in 20000 100000 140000 200000; do
  timeout -k 10 300 python bench.py --workload stream --qps $q --duration 2 > gpurun_out/${TAG}_stream_$q.log 2>&1 || exit $?
  echo "stream $q: $(j gpurun_out/${TAG}_stream_$q.log 'round(d["value"]), round(d["p50_ms"],2), round(d["p99_ms"],2), round(d["mean_batch"],1)')"
done
timeout -k 10 300 python bench.py --workload stream --max-batch 512 --qps 320000 --duration 1.5 > gpurun_out/${TAG}_stream_b512.log 2>&1 || exit $?
echo "stream b512 320k: $(j gpurun_out/${TAG}_stream_b512.log 'round(d["value"]), round(d["p50_ms"],2), round(d["p99_ms"],2), round(d["mean_batch"],1)')"
for q in 20000 60000; do
  timeout -k 10 300 python bench.py --workload stream --search-type hybrid --qps $q --duration 2 > gpurun_out/${TAG}_stream_hyb_$q.log 2>&1 || exit $?
  echo "stream hybrid $q: $(j gpurun_out/${TAG}_stream_hyb_$q.log 'round(d["value"]), round(d["p50_ms"],2), round(d["p99_ms"],2), round(d["mean_batch"],1)')"
done
timeout -k 10 600 python bench.py --workload pipeline --queries 100 > gpurun_out/${TAG}_bench_pipeline.log 2>&1 || exit $?
echo "pipeline: $(tail -1 gpurun_out/${TAG}_bench_pipeline.log | cut -c1-220)"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --latency-iters 2"
P="$R/gpurun_out/${TAG}_p"; mkdir -p "$P"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$P/dense" -o run -- python3 $B > "$P/dense.log" 2>&1 || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$P/rerank" -o run -- python3 $R/bench.py --workload hybrid_rerank --steps 3 --warmup 1 --latency-iters 1 --no-cpu-baseline > "$P/rerank.log" 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$P/fetch" -o run -- python3 $B > "$P/fetch.log" 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$P/write" -o run -- python3 $B > "$P/write.log" 2>&1 || exit $?
# keep the summaries only (gpurun copies back at most 64 MiB)
python3 "$R/tools/rocpd_stats.py" "$P/dense/run_results.db" > "$R/gpurun_out/${TAG}_dense_kernel_stats.csv" || exit $?
python3 "$R/tools/rocpd_stats.py" "$P/rerank/run_results.db" > "$R/gpurun_out/${TAG}_rerank_kernel_stats.csv" || exit $?
python3 "$R/tools/pmc_traffic.py" "$P/fetch/run_counter_collection.csv" "$P/write/run_counter_collection.csv" "dense_scan_i8_kernel<1024, false, false>" 1032131072 "bench.py default: 1M x 1024 rows, int8 filter image (tile-blocked, scattered row order) + a32/e32, 64 fp16 queries per launch" > "$R/gpurun_out/${TAG}_dense_scan_i8_traffic.json" || exit $?
rm -rf "$P"
echo "profiles done"
