#!/bin/bash
# Round 3: intra-workgroup tile counter in the int8 scan: parity, bench (1M k5/k40, 100k), stamps.
TAG=${1:-r03j}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
j() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($2)"; }
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_dense_gpu.py tests/test_dense_collect_gpu.py tests/test_dense_filter_gpu.py tests/test_fullsize_gpu.py \
  > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
B="--no-extras --no-cpu-baseline --latency-iters 3"
for rep in 1 2; do
  for args in "" "--top-k 40" "--chunks 100000 --steps 200"; do
    n=$(echo "$rep $args" | tr ' -' '__')
    timeout -k 10 200 python bench.py $B $args > gpurun_out/${TAG}_$n.log 2>&1 || exit $?
    echo "#$rep [$args]: $(j gpurun_out/${TAG}_$n.log 'round(d["value"]), round(d["ms_per_step"],4), round(d["roofline"]["avg_launch_ms"],4), d["certified_frac"]')"
  done
done
bash tools/probes/i8_stamps.sh ${TAG}stp || exit $?
