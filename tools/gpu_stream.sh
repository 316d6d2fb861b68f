#!/bin/bash
# Streaming front ends: GPU tests (oracle parity), then the stream workload at several offered
# rates (native server + native load generator) and the Python front end for comparison.
TAG=${1:-st}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_batcher_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
for q in ${QPS:-20000 60000 100000 140000}; do
  timeout -k 10 300 python bench.py --workload stream --qps $q --duration 3 > gpurun_out/${TAG}_native_$q.log 2>&1 || exit $?
  echo "native $q: $(tail -1 gpurun_out/${TAG}_native_$q.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["p50_ms"],2), round(d["p99_ms"],2), round(d["mean_batch"],1))')"
done
timeout -k 10 300 python bench.py --workload stream --stream-front python --qps 20000 --duration 3 > gpurun_out/${TAG}_python_20000.log 2>&1 || exit $?
echo "python 20000: $(tail -1 gpurun_out/${TAG}_python_20000.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["p50_ms"],2), round(d["p99_ms"],2), round(d["mean_batch"],1))')"
timeout -k 10 400 python bench.py --workload ingest --ingest-chunks 20000 --qps 50000 --duration 2 > gpurun_out/${TAG}_ingest.log 2>&1 || exit $?
echo "ingest: $(tail -1 gpurun_out/${TAG}_ingest.log | cut -c1-100) $(tail -1 gpurun_out/${TAG}_ingest.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["embed_chunks_per_s"], d["index_chunks_per_s"], round(d["p99_ms"],2))')"
