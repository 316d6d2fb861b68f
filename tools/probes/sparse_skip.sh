#!/bin/bash
# Sparse scan with active-term skipping: sparse / hybrid parity tests, then the hybrid bench.
TAG=${1:-sk}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sparse_rrf_gpu.py tests/test_fullsize_gpu.py tests/test_golden_pipeline_gpu.py tests/test_batcher_gpu.py \
  -k "not bge and not rerank and not shard_scan" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload hybrid --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_hybrid$i.log 2>&1 || exit $?
  echo "hybrid: $(tail -1 gpurun_out/${TAG}_hybrid$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],3), d["roofline_sparse"]["avg_launch_ms"])')"
done
