#!/bin/bash
# Round-3: int8 scan without the per-tile prefetch drain; static vs dynamic (asm dequeue),
# parity of both schedules, phase stamps of both.
TAG=${1:-r03g}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
j() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($2)"; }
for sched in static dynamic; do
  ARMI_I8_SCHED=$sched timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_dense_gpu.py tests/test_dense_collect_gpu.py tests/test_dense_filter_gpu.py \
    > gpurun_out/${TAG}_pytest_$sched.log 2>&1; rc=$?
  echo "pytest $sched rc=$rc $(tail -1 gpurun_out/${TAG}_pytest_$sched.log)"
  [ $rc -eq 0 ] || exit $rc
done
B="--no-extras --no-cpu-baseline --latency-iters 3"
for rep in 1 2; do
  for sched in static dynamic; do
    for args in "" "--top-k 40" "--chunks 100000 --steps 200"; do
      n=$(echo "$sched $rep $args" | tr ' -' '__')
      ARMI_I8_SCHED=$sched timeout -k 10 200 python bench.py $B $args > gpurun_out/${TAG}_$n.log 2>&1 || exit $?
      echo "$sched #$rep [$args]: $(j gpurun_out/${TAG}_$n.log 'round(d["value"]), round(d["ms_per_step"],4), round(d["roofline"]["avg_launch_ms"],4), d["certified_frac"]')"
    done
  done
done
ARMI_DENSE_FILTER=fp16 timeout -k 10 200 python bench.py $B > gpurun_out/${TAG}_fp16pass.log 2>&1 || exit $?
echo "fp16 pass: $(j gpurun_out/${TAG}_fp16pass.log 'round(d["value"]), round(d["ms_per_step"],4), round(d["roofline"]["avg_launch_ms"],4), d["roofline"]["kernel"]')"
ARMI_I8_SCHED=static bash tools/probes/i8_stamps.sh ${TAG}stps || exit $?
ARMI_I8_SCHED=dynamic bash tools/probes/i8_stamps.sh ${TAG}stpd || exit $?

