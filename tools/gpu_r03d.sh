#!/bin/bash
# Round-3: dynamic tile schedule of the int8 scan. Dense parity tests, headline A/B (dynamic vs
# static split), k = 40 and configs[1] shapes, and the phase stamps of the dynamic form.
TAG=${1:-r03d}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
j() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($2)"; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_dense_gpu.py tests/test_dense_collect_gpu.py tests/test_dense_filter_gpu.py tests/test_batcher_gpu.py \
  > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
B="--no-extras --no-cpu-baseline --latency-iters 3"
for mode in "dynamic 2" "dynamic 1" "static 1"; do
  set -- $mode
  for args in "" "--top-k 40" "--chunks 100000 --steps 200"; do
    n=$(echo "$1 p$2 $args" | tr ' -' '__')
    ARMI_I8_SCHED=$1 timeout -k 10 200 python bench.py $B --pipeline $2 $args > gpurun_out/${TAG}_$n.log 2>&1 || exit $?
    echo "$1 pipe$2 [$args]: $(j gpurun_out/${TAG}_$n.log 'round(d["value"]), round(d["ms_per_step"],4), round(d["roofline"]["avg_launch_ms"],4), d["certified_frac"]')"
  done
done
bash tools/probes/i8_stamps.sh ${TAG}stp
