#!/bin/bash
# Round 3: branch-free wave sorts + padded merge rows: full -m gpu suite, dense bench x2, hybrid,
# stamps.
TAG=${1:-r03l}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
j() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($2)"; }
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
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
timeout -k 10 300 python bench.py --workload hybrid --no-cpu-baseline --latency-iters 3 > gpurun_out/${TAG}_hybrid.log 2>&1 || exit $?
echo "hybrid: $(j gpurun_out/${TAG}_hybrid.log 'round(d["value"]), round(d["ms_per_step"],4), round(d["roofline_sparse"]["avg_launch_ms"],4)')"
bash tools/probes/i8_stamps.sh ${TAG}stp || exit $?
