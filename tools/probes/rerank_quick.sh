#!/bin/bash
# Cross-encoder parity tests and the hybrid_rerank bench (after encoder-kernel changes).
TAG=${1:-rq}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_encoder_gpu.py tests/test_fullsize_gpu.py -k "encoder or rerank or cross or head" \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --workload hybrid_rerank --steps 5 --warmup 2 --latency-iters 2 --no-cpu-baseline > gpurun_out/${TAG}_rerank.log 2>&1 || exit $?
echo "rerank: $(tail -1 gpurun_out/${TAG}_rerank.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["ms_per_step"],2), d["roofline"]["avg_forward_ms"], round(d["roofline"]["frac"],3))')"
