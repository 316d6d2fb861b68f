#!/bin/bash
# Two-stage merge rescore: dense parity suites, then bench A/B (ARMI_MERGE_RESCORE=exact) at k 5 /
# 40 and 100k, and the hybrid step.
TAG=${1:-r03y}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
j() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($2)"; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_dense_gpu.py tests/test_dense_filter_gpu.py tests/test_dense_collect_gpu.py \
  tests/test_fullsize_gpu.py tests/test_store_gpu.py tests/test_golden_pipeline_gpu.py \
  > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
B="--no-extras --no-cpu-baseline --latency-iters 5"
for rep in 1 2; do
  for mode in two exact; do
    if [ $mode = exact ]; then export ARMI_MERGE_RESCORE=exact; else unset ARMI_MERGE_RESCORE; fi
    for args in "" "--top-k 40" "--chunks 100000 --steps 200"; do
      n=$(echo "$mode $rep $args" | tr ' -' '__')
      timeout -k 10 200 python bench.py $B $args > gpurun_out/${TAG}_$n.log 2>&1 || exit $?
      echo "$mode #$rep [$args]: $(j gpurun_out/${TAG}_$n.log 'round(d["value"]), round(d["ms_per_step"],4), round(d["p50_ms"],3), d["certified_frac"]')"
    done
    timeout -k 10 300 python bench.py --workload hybrid $B > gpurun_out/${TAG}_hyb_${mode}_$rep.log 2>&1 || exit $?
    echo "$mode #$rep hybrid: $(j gpurun_out/${TAG}_hyb_${mode}_$rep.log 'round(d["value"]), round(d["ms_per_step"],4)')"
  done
done
unset ARMI_MERGE_RESCORE
cd /tmp && export TMPDIR=/tmp
P="$R/gpurun_out/${TAG}_p"; mkdir -p "$P"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$P/dense" -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --latency-iters 2 > "$P/dense.log" 2>&1 || exit $?
python3 "$R/tools/rocpd_stats.py" "$P/dense/run_results.db" > "$R/gpurun_out/${TAG}_dense_kernel_stats.csv" || exit $?
rm -rf "$P"
grep -E "merge|scan_i8" "$R/gpurun_out/${TAG}_dense_kernel_stats.csv" | cut -c1-40,120-200
