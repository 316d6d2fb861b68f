#!/bin/bash
# fp16 -> 2^24 fixed point through fp32 (3 instructions): parity of every exact path, then bench A/B
# against the previous build (ablibs/libarmi_prev.so) at 1M (k 5, 40) and 100k.
TAG=${1:-r03aa}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
j() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($2)"; }
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_dense_gpu.py tests/test_dense_filter_gpu.py tests/test_dense_collect_gpu.py \
  tests/test_fullsize_gpu.py tests/test_store_gpu.py tests/test_shards_gpu.py tests/test_golden_pipeline_gpu.py \
  > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
B="--no-extras --no-cpu-baseline --latency-iters 5"
for rep in 1 2; do
  for lib in new prev; do
    if [ $lib = prev ]; then export ARMI_LIB_PATH=ablibs/libarmi_prev.so; else unset ARMI_LIB_PATH; fi
    for args in "" "--top-k 40" "--chunks 100000 --steps 200"; do
      n=$(echo "$lib $rep $args" | tr ' -' '__')
      timeout -k 10 200 python bench.py $B $args > gpurun_out/${TAG}_$n.log 2>&1 || exit $?
      echo "$lib #$rep [$args]: $(j gpurun_out/${TAG}_$n.log 'round(d["value"]), round(d["ms_per_step"],4), round(d["p50_ms"],3), d["certified_frac"]')"
    done
  done
done
