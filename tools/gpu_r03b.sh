#!/bin/bash
# Round-3 validation session: the full -m gpu suite, smoke, the dense headline, native stream
# benches (the stream server changed: lifetime, ring sizing, concurrent loadgen collector).
TAG=${1:-r03b}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
j() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($2)"; }
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
echo "smoke ok"
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench_dense.log 2>&1 || exit $?
echo "dense: $(j gpurun_out/${TAG}_bench_dense.log 'round(d["value"]), round(d["ms_per_step"],4), d["roofline"]["kernel"], round(d["roofline"]["frac"],3), round(d["cpu_baseline"]["value"],1)')"
for q in 100000 200000; do
  timeout -k 10 300 python bench.py --workload stream --qps $q --duration 2 > gpurun_out/${TAG}_stream_$q.log 2>&1 || exit $?
  echo "stream $q: $(j gpurun_out/${TAG}_stream_$q.log 'round(d["value"]), round(d["p50_ms"],2), round(d["p99_ms"],2), round(d["mean_batch"],1)')"
done
timeout -k 10 300 python bench.py --workload stream --search-type hybrid --qps 60000 --duration 2 > gpurun_out/${TAG}_stream_hyb.log 2>&1 || exit $?
echo "stream hybrid 60k: $(j gpurun_out/${TAG}_stream_hyb.log 'round(d["value"]), round(d["p50_ms"],2), round(d["p99_ms"],2)')"
timeout -k 10 600 python bench.py --workload hybrid_rerank --steps 5 --warmup 2 --latency-iters 3 --no-cpu-baseline > gpurun_out/${TAG}_bench_rerank.log 2>&1 || exit $?
echo "rerank: $(j gpurun_out/${TAG}_bench_rerank.log 'round(d["value"],1), round(d["ms_per_step"],2), round(d["roofline"]["frac"],3), round(d["roofline_scan"]["avg_launch_ms"],4), d["roofline_scan"]["kernel"]')"
echo done
