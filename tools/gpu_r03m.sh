#!/bin/bash
# Round 3: precomputed query image A/B (DMA vs in-kernel build), same box; parity; stamps.
TAG=${1:-r03m}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
j() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($2)"; }
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_dense_gpu.py tests/test_dense_collect_gpu.py tests/test_dense_filter_gpu.py \
  > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
B="--no-extras --no-cpu-baseline --latency-iters 3"
for rep in 1 2; do
  for img in dma inkernel; do
    for args in "" "--chunks 100000 --steps 200"; do
      n=$(echo "$img $rep $args" | tr ' -' '__')
      ARMI_I8_IMAGE=$img timeout -k 10 200 python bench.py $B $args > gpurun_out/${TAG}_$n.log 2>&1 || exit $?
      echo "$img #$rep [$args]: $(j gpurun_out/${TAG}_$n.log 'round(d["value"]), round(d["ms_per_step"],4), round(d["roofline"]["avg_launch_ms"],4), d["certified_frac"]')"
    done
  done
done
bash tools/probes/i8_stamps.sh ${TAG}stp || exit $?
