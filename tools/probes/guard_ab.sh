#!/bin/bash
# Parity with the insert guard (default), then A/B of ARMI_INSERT_GUARD=0/1: per-GPU compute of
# the sharded step (G = 1, 2, 4, 8 at 1M chunks; G = 8 at 10M) and the headline bench line.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dense_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/guard_tests.log 2>&1; rc=$?
tail -2 gpurun_out/guard_tests.log
[ $rc -eq 0 ] || exit $rc
for g in 0 1 0 1; do
  ARMI_INSERT_GUARD=$g timeout -k 10 200 python tools/shard_bench.py > gpurun_out/guard_sb_$g.log 2>&1 || exit $?
  echo "guard=$g"; tail -4 gpurun_out/guard_sb_$g.log
done
for g in 0 1; do
  ARMI_INSERT_GUARD=$g timeout -k 10 300 python tools/shard_bench.py --gs 8 --chunks 10000000 > gpurun_out/guard_sb10m_$g.log 2>&1 || exit $?
  echo "10M guard=$g $(tail -1 gpurun_out/guard_sb10m_$g.log)"
done
for g in 0 1 0 1; do
  ARMI_INSERT_GUARD=$g timeout -k 10 300 python bench.py > gpurun_out/guard_bench_$g.json 2> gpurun_out/guard_bench_$g.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/guard_bench_$g.json')); print('bench guard=$g', round(d['value']), d['roofline']['avg_launch_ms'], round(d['roofline']['frac'],3))"
done
