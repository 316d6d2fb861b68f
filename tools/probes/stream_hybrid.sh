#!/bin/bash
# Batcher / native stream server parity (dense + hybrid), cls-head encoder checks, then the
# hybrid native stream bench at a few offered rates.
TAG=${1:-sh}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_batcher_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_batcher.log 2>&1; rc=$?
echo "batcher rc=$rc $(tail -1 gpurun_out/${TAG}_batcher.log)"
[ $rc -eq 0 ] || exit $rc
bash tools/probes/rerank_quick.sh ${TAG} || exit $?
for q in ${QPS:-20000 60000 100000}; do
  timeout -k 10 300 python bench.py --workload stream --search-type hybrid --qps $q --duration 1.5 \
    > gpurun_out/${TAG}_hyb_${q}.log 2>&1 || exit $?
  echo "hybrid $q: $(tail -1 gpurun_out/${TAG}_hyb_${q}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["p50_ms"],2), round(d["p99_ms"],2), round(d["mean_batch"],1))')"
done
