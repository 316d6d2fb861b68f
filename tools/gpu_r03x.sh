#!/bin/bash
# RRF by counting: parity (sparse / RRF / batcher / golden pipeline tests), the hybrid step's kernel
# stats + timeline, then the driver's default bench line.
TAG=${1:-r03x}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_sparse_rrf_gpu.py tests/test_batcher_gpu.py tests/test_golden_pipeline_gpu.py \
  > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
j() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($2)"; }
timeout -k 10 300 python bench.py --workload hybrid --no-cpu-baseline > gpurun_out/${TAG}_bench_hybrid.log 2>&1 || exit $?
echo "hybrid: $(j gpurun_out/${TAG}_bench_hybrid.log 'round(d["value"]), round(d["ms_per_step"],4)')"
ARMI_HYBRID_ORDER=dense timeout -k 10 300 python bench.py --workload hybrid --no-cpu-baseline > gpurun_out/${TAG}_bench_hybrid_dfirst.log 2>&1 || exit $?
echo "hybrid dense-first: $(j gpurun_out/${TAG}_bench_hybrid_dfirst.log 'round(d["value"]), round(d["ms_per_step"],4)')"
ARMI_HYBRID_SERIAL=1 timeout -k 10 300 python bench.py --workload hybrid --no-cpu-baseline > gpurun_out/${TAG}_bench_hybrid_serial.log 2>&1 || exit $?
echo "hybrid serial: $(j gpurun_out/${TAG}_bench_hybrid_serial.log 'round(d["value"]), round(d["ms_per_step"],4)')"
bash tools/probes/hyb_stats.sh ${TAG} > gpurun_out/${TAG}_hybst.txt 2>&1 || exit $?
grep -i "rrf" gpurun_out/${TAG}_hybrid_kernel_stats.csv | cut -c1-30,60-140
bash tools/gpu_bench_default.sh ${TAG}
