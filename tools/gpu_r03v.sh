#!/bin/bash
# CU-split pipelined dense step (scan on the scan stream's CUs, merge on reserved CUs): parity
# test, then bench A/B against the one-batch step and the two-stream pipeline, same box.
TAG=${1:-r03v}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
j() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($2)"; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_dense_gpu.py > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
B="--no-extras --no-cpu-baseline --latency-iters 5"
for rep in 1 2; do
  for mode in "p1" "m8" "m16" "m4"; do
    case $mode in
      p1) a="";; p2) a="--pipeline 2";; m8) a="--pipeline 2 --merge-cus 8";;
      m16) a="--pipeline 2 --merge-cus 16";; m4) a="--pipeline 2 --merge-cus 4";;
    esac
    for sz in "" "--chunks 100000 --steps 200"; do
      n=$(echo "$mode $rep $sz" | tr ' -' '__')
      timeout -k 10 200 python bench.py $B $a $sz > gpurun_out/${TAG}_$n.log 2>&1 || exit $?
      echo "$mode #$rep [$sz]: $(j gpurun_out/${TAG}_$n.log 'round(d["value"]), round(d["ms_per_step"],4), round(d["p50_ms"],3), round(d["roofline"]["avg_launch_ms"],4), d["certified_frac"]')"
    done
  done
done
