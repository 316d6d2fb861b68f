#!/bin/bash
# Round 3: sparse scan clearing only dirty staged rows (A/B vs ARMI_SPARSE_CLEAR=all), parity;
# int8-scan PMC traffic (first pass only) + stamps with per-workgroup spreads.
TAG=${1:-r03i}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
j() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($2)"; }
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_sparse_rrf_gpu.py tests/test_batcher_gpu.py tests/test_store_gpu.py \
  > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for c in dirty all; do
    ARMI_SPARSE_CLEAR=$c timeout -k 10 300 python bench.py --workload hybrid --no-cpu-baseline --latency-iters 3 > gpurun_out/${TAG}_hyb_${c}_$rep.log 2>&1 || exit $?
    echo "hybrid clear=$c #$rep: $(j gpurun_out/${TAG}_hyb_${c}_$rep.log 'round(d["value"]), round(d["ms_per_step"],4), round(d["roofline_sparse"]["avg_launch_ms"],4)')"
  done
done
bash tools/gpu_pmc_i8.sh ${TAG}pmc || exit $?
cd "$R" && bash tools/probes/i8_stamps.sh ${TAG}stp || exit $?
