#!/bin/bash
# Int8 scan prologue change: dense parity (dense, filter, full-size), then dense bench at 1M and 10M.
TAG=${1:-pro}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_dense_gpu.py tests/test_dense_filter_gpu.py tests/test_fullsize_gpu.py tests/test_golden_pipeline_gpu.py -k "not bge and not rerank" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
for n in 1000000 1000000 10000000; do
  timeout -k 10 400 python bench.py --chunks $n --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 10 > gpurun_out/${TAG}_$n.log 2>&1 || exit $?
  echo "$n: $(tail -1 gpurun_out/${TAG}_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]), round(d["ms_per_step"],4), "p50", round(d["p50_ms"],4), "scan", round(r["avg_launch_ms"],4), round(r["frac"],3), d["certified_frac"])')"
done
