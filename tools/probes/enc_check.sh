#!/bin/bash
# armi batch-1 query encoder: the full -m gpu suite, then the pipeline workload
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out || exit 1
TAG=${1:-enc}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -1 gpurun_out/${TAG}_pytest.log; grep -E "^FAILED|Error" gpurun_out/${TAG}_pytest.log | head -10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
grep -E "bge-m3 24 layers" gpurun_out/${TAG}_pytest.log | head -8
timeout -k 10 400 python bench.py --workload pipeline --queries 200 > gpurun_out/${TAG}_pipeline.json 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_pipeline.json').read().strip().splitlines()[-1]);print('pipeline p50',round(d['p50_ms'],3),'p99',round(d['p99_ms'],3),d['stage_p50_ms'],'q/s',round(d['value'],1))"
