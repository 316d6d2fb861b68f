#!/bin/bash
# Round-3 dense second pass: collect / scattered-image tests, then dense benches on the random and
# the clustered corpus at k = 5 and k = 40 (no CPU baseline), one rocprofv3 kernel-stats run.
TAG=${1:-r03a}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
j() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($2)"; }
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_dense_collect_gpu.py tests/test_dense_filter_gpu.py tests/test_dense_gpu.py \
  > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
B="--no-cpu-baseline --latency-iters 5 --steps 40"
for c in random clustered; do
  for k in 5 40; do
    timeout -k 10 300 python bench.py $B --corpus $c --top-k $k > gpurun_out/${TAG}_dense_${c}_k$k.log 2>&1 || exit $?
    echo "$c k=$k: $(j gpurun_out/${TAG}_dense_${c}_k$k.log 'round(d["value"]), round(d["ms_per_step"],4), d["certified_frac"], d["roofline"]["kernel"], round(d["roofline"]["avg_launch_ms"],4)')"
  done
done
cd /tmp && export TMPDIR=/tmp
P="$R/gpurun_out/${TAG}_p"; mkdir -p "$P"
for c in random clustered; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$P/$c" -o run -- python3 $R/bench.py $B --corpus $c > "$P/$c.log" 2>&1 || exit $?
python3 "$R/tools/rocpd_stats.py" "$P/$c/run_results.db" > "$R/gpurun_out/${TAG}_${c}_kernel_stats.csv" || exit $?
done
rm -rf "$P"
echo done
