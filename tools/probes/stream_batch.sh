#!/bin/bash
# Native streaming server: offered rate beyond the 64-query scan's capacity with larger batches.
TAG=${1:-sb}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
for mb_q in 64:160000 64:200000 128:200000 256:200000 256:260000 512:260000 512:320000; do
  mb=${mb_q%%:*}; q=${mb_q##*:}
  timeout -k 10 300 python bench.py --workload stream --qps $q --duration 1.5 --max-batch $mb > gpurun_out/${TAG}_${mb}_$q.log 2>&1 || exit $?
  echo "max_batch $mb offered $q: $(tail -1 gpurun_out/${TAG}_${mb}_$q.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["p50_ms"],2), round(d["p99_ms"],2), round(d["mean_batch"],1))')"
done
