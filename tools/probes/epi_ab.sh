#!/bin/bash
# Dense/filter parity after the epilogue change, then per-GPU compute of the sharded step
# (G = 1..8 at 1M, G = 8 at 10M) and the headline bench line.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_dense_gpu.py tests/test_golden_pipeline_gpu.py tests/test_store_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/epi_tests.log 2>&1; rc=$?
tail -2 gpurun_out/epi_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/shard_bench.py > gpurun_out/epi_sb.log 2>&1 || exit $?
tail -4 gpurun_out/epi_sb.log
for st in reg glds; do
  ARMI_GEMM_STAGE=$st timeout -k 10 300 python tools/shard_bench.py --gs 8 --chunks 10000000 > gpurun_out/epi_sb10m_$st.log 2>&1 || exit $?
  echo "10M stage=$st $(tail -1 gpurun_out/epi_sb10m_$st.log)"
done
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/epi_bench_$i.json 2> gpurun_out/epi_bench_$i.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/epi_bench_$i.json')); print('bench', round(d['value']), d['roofline']['avg_launch_ms'], round(d['roofline']['frac'],3))"
done
