#!/bin/bash
# Round 3 (session 2): cross-encoder A/B: attention VALU cut + A&S GELU epilogue vs the r03n build
# (ablibs/libarmi_head.so); parity of the encoder / GEMM kernels and the 12-layer rerank.
TAG=${1:-r03o}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
j() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($2)"; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gemm_gpu.py tests/test_encoder_gpu.py "tests/test_fullsize_gpu.py::test_configs2_rerank_full_depth_within_1e3" \
  > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/probes/gemm_bench.py > gpurun_out/${TAG}_gemm_new.log 2>&1 || exit $?
ARMI_LIB_PATH=ablibs/libarmi_head.so timeout -k 10 200 python -u tools/probes/gemm_bench.py > gpurun_out/${TAG}_gemm_head.log 2>&1 || exit $?
echo new; cat gpurun_out/${TAG}_gemm_new.log; echo head; cat gpurun_out/${TAG}_gemm_head.log
timeout -k 10 200 python -u tools/probes/attention_time.py > gpurun_out/${TAG}_att_oneshot.log 2>&1 || exit $?
ARMI_ATTENTION=persist timeout -k 10 200 python -u tools/probes/attention_time.py > gpurun_out/${TAG}_att_persist.log 2>&1 || exit $?
echo oneshot; grep n= gpurun_out/${TAG}_att_oneshot.log; echo persist; grep n= gpurun_out/${TAG}_att_persist.log
B="--workload hybrid_rerank --no-extras --no-cpu-baseline --steps 10 --warmup 3"
for rep in 1 2; do
  for lib in new head; do
    if [ $lib = head ]; then export ARMI_LIB_PATH=ablibs/libarmi_head.so; else unset ARMI_LIB_PATH; fi
    timeout -k 10 300 python bench.py $B > gpurun_out/${TAG}_rerank_${lib}_$rep.log 2>&1 || exit $?
    echo "$lib #$rep: $(j gpurun_out/${TAG}_rerank_${lib}_$rep.log 'round(d["value"],1), round(d["ms_per_step"],3), d["roofline"]["achieved"]')"
  done
done
