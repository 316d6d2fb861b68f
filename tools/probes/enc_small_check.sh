#!/bin/bash
# small-M encoder linears: parity (GEMM, encoder, full-depth BGE-M3, query graphs), pipeline, profile
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out || exit 1
TAG=${1:-esm}
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gemm_gpu.py tests/test_encoder_gpu.py tests/test_query_graph_gpu.py "tests/test_fullsize_gpu.py::test_bge_m3_full_depth_matches_fp32" > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -1 gpurun_out/${TAG}_pytest.log; grep -E "^FAILED" gpurun_out/${TAG}_pytest.log | head -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --workload pipeline --queries 200 > gpurun_out/${TAG}_pipeline.json 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_pipeline.json').read().strip().splitlines()[-1]);print('pipeline p50',round(d['p50_ms'],3),'p99',round(d['p99_ms'],3),d['stage_p50_ms'],'q/s',round(d['value'],1))"
bash tools/probes/embed_prof.sh ${TAG}_ep
