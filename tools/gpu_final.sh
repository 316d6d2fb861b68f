#!/bin/bash
# Round-end measurement session: full -m gpu suite (as the driver runs it), every bench
# workload, kernel-trace stats of the dense and rerank benches, and the dense scan's HBM traffic
# (FETCH_SIZE / WRITE_SIZE passes, one counter group per run). Each GPU step has its own limit;
# a crash / timeout ends the session.
TAG=${1:-final}
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 1
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc: $(tail -1 gpurun_out/${TAG}_pytest.log)"
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
echo "smoke: $(tail -1 gpurun_out/${TAG}_smoke.log)"
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench_dense.log 2>&1 || exit $?
echo "dense done"
timeout -k 10 300 python bench.py --workload hybrid --steps 20 --warmup 3 > gpurun_out/${TAG}_bench_hybrid.log 2>&1 || exit $?
echo "hybrid done"
timeout -k 10 400 python bench.py --workload hybrid_rerank --steps 5 --warmup 2 --latency-iters 3 \
  > gpurun_out/${TAG}_bench_rerank.log 2>&1 || exit $?
echo "rerank done"
timeout -k 10 300 python bench.py --workload stream --qps 10000 --duration 3 > gpurun_out/${TAG}_bench_stream.log 2>&1 || exit $?
echo "stream done"
timeout -k 10 500 python bench.py --workload pipeline --queries 200 > gpurun_out/${TAG}_bench_pipeline.log 2>&1 || exit $?
echo "pipeline done"
timeout -k 10 300 python tools/shard_bench.py > gpurun_out/${TAG}_shard.log 2>&1 || exit $?
echo "shard done"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --latency-iters 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_prof_dense" -o run -- \
  python3 $B > "$R/gpurun_out/${TAG}_prof_dense.log" 2>&1 || exit $?
echo "prof dense done"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_prof_rerank" -o run -- \
  python3 "$R/bench.py" --workload hybrid_rerank --steps 3 --warmup 1 --latency-iters 1 > "$R/gpurun_out/${TAG}_prof_rerank.log" 2>&1 || exit $?
echo "prof rerank done"
P="$R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --latency-iters 2"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/${TAG}_fetch" -o run -- python3 $P > "$R/gpurun_out/${TAG}_fetch.log" 2>&1 || exit $?
echo "fetch done"
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/${TAG}_write" -o run -- python3 $P > "$R/gpurun_out/${TAG}_write.log" 2>&1 || exit $?
echo "write done"
exit 0
