#!/bin/bash
# Sparse merge: one-round pool loads + radix-selected t0 + one-wave sorts. Parity (sparse, RRF,
# shards, full-size hybrid, golden, batcher), hybrid bench A/B vs the previous build, kernel stats.
TAG=${1:-r03ab}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
j() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($2)"; }
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_sparse_rrf_gpu.py tests/test_shards_gpu.py tests/test_batcher_gpu.py \
  tests/test_golden_pipeline_gpu.py tests/test_ingest_stream_gpu.py \
  "tests/test_fullsize_gpu.py::test_configs2_hybrid_1m_matches_oracle" \
  "tests/test_fullsize_gpu.py::test_configs3_hybrid_shards_match_oracle" \
  > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
B="--workload hybrid --no-cpu-baseline --latency-iters 5"
for rep in 1 2 3; do
  for lib in new prev; do
    if [ $lib = prev ]; then export ARMI_LIB_PATH=ablibs/libarmi_prev.so; else unset ARMI_LIB_PATH; fi
    timeout -k 10 300 python bench.py $B > gpurun_out/${TAG}_${lib}_$rep.log 2>&1 || exit $?
    echo "$lib #$rep hybrid: $(j gpurun_out/${TAG}_${lib}_$rep.log 'round(d["value"]), round(d["ms_per_step"],4)')"
  done
done
unset ARMI_LIB_PATH
bash tools/probes/hyb_stats.sh ${TAG} > /dev/null 2>&1 || exit $?
grep -E "sparse_merge|dense_merge|rrf_kernel|pass_terms" gpurun_out/${TAG}_hybrid_kernel_stats.csv | cut -c1-45,150-220
