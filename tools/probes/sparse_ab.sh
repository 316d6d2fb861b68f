#!/bin/bash
# Sparse scan change: sparse / hybrid parity, then the hybrid bench (sparse scan time, step).
TAG=${1:-sp}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_sparse_rrf_gpu.py tests/test_fullsize_gpu.py tests/test_batcher_gpu.py tests/test_golden_pipeline_gpu.py -k "not bge and not rerank" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 400 python bench.py --workload hybrid --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 5 > gpurun_out/${TAG}_hyb$i.log 2>&1 || exit $?
  echo "hybrid: $(tail -1 gpurun_out/${TAG}_hyb$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["roofline_sparse"]; print(round(d["value"]), round(d["ms_per_step"],3), "sparse_ms", round(s["avg_launch_ms"],4), round(s["achieved"]))')"
done
timeout -k 10 300 python tools/sparse_bench.py --iters 100 > gpurun_out/${TAG}_sb.log 2>&1 || exit $?
echo "sparse alone: $(tail -1 gpurun_out/${TAG}_sb.log)"
