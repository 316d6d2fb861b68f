#!/bin/bash
# A/B: hybrid bench with the new and the old library, then the sparse/RRF GPU tests (new).
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
L=audio_rag_amd/_lib
cp $L/libarmi.so $L/libarmi_new.so
for v in new old new old; do
  cp $L/libarmi_$v.so $L/libarmi.so
  timeout -k 10 200 python bench.py --workload hybrid --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]);print('$v', round(d['value']), d['ms_per_step'])"
done
cp $L/libarmi_new.so $L/libarmi.so
timeout -k 10 300 python -u -m pytest tests/test_sparse_rrf_gpu.py tests/test_golden_pipeline_gpu.py tests/test_store_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1; rc=$?
tail -2 gpurun_out/ab_tests.log; exit $rc
