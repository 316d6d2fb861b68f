#!/bin/bash
# Round-3 validation session: the full -m gpu suite, smoke, the dense headline (+ configs1 /
# configs2 extras), the clustered corpus, a kernel-trace profile of the headline, native stream
# benches, and the rerank attention A/B (persistent vs one-shot) on the mixed GEMM default.
TAG=${1:-r03b}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
export TMPDIR=/tmp
j() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($2)"; }
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
echo "smoke ok"
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench_dense.log 2>&1 || exit $?
echo "dense: $(j gpurun_out/${TAG}_bench_dense.log 'round(d["value"]), round(d["ms_per_step"],4), d["roofline"]["kernel"], round(d["roofline"]["frac"],3), round(d["cpu_baseline"]["value"],1)')"
echo "configs1: $(j gpurun_out/${TAG}_bench_dense.log 'round(d["configs1"]["value"]), round(d["configs1"]["ms_per_step"],4)')"
echo "configs2: $(j gpurun_out/${TAG}_bench_dense.log 'round(d["configs2"]["value"],1), round(d["configs2"]["ms_per_step"],2), round(d["configs2"]["roofline_scan"]["avg_launch_ms"],4)')"
timeout -k 10 300 python bench.py --corpus clustered --no-extras --no-cpu-baseline > gpurun_out/${TAG}_bench_clustered.log 2>&1 || exit $?
echo "clustered: $(j gpurun_out/${TAG}_bench_clustered.log 'round(d["value"]), round(d["ms_per_step"],4), d["certified_frac"]')"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof" -o dense -- python3 "$R/bench.py" --no-extras --no-cpu-baseline --steps 50 > "$R/gpurun_out/${TAG}_prof.log" 2>&1 || exit $?
cd "$R"
for q in 100000 200000; do
  timeout -k 10 300 python bench.py --workload stream --qps $q --duration 2 > gpurun_out/${TAG}_stream_$q.log 2>&1 || exit $?
  echo "stream $q: $(j gpurun_out/${TAG}_stream_$q.log 'round(d["value"]), round(d["p50_ms"],2), round(d["p99_ms"],2), round(d["mean_batch"],1)')"
done
RR="--workload hybrid_rerank --steps 4 --warmup 2 --latency-iters 1 --no-cpu-baseline"
timeout -k 10 400 python bench.py $RR > gpurun_out/${TAG}_rerank.log 2>&1 || exit $?
echo "rerank mixed+persist: $(j gpurun_out/${TAG}_rerank.log 'round(d["value"],1), round(d["roofline"]["avg_forward_ms"],2), round(d["roofline"]["frac"],3), round(d["roofline_scan"]["avg_launch_ms"],4)')"
ARMI_ATTENTION=oneshot timeout -k 10 400 python bench.py $RR > gpurun_out/${TAG}_rerank_oneshot.log 2>&1 || exit $?
echo "rerank mixed+oneshot: $(j gpurun_out/${TAG}_rerank_oneshot.log 'round(d["value"],1), round(d["roofline"]["avg_forward_ms"],2)')"
echo done
