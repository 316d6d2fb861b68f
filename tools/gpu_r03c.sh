#!/bin/bash
# Round-3: GEMM parity + speed vs hipBLASLt, encoder tests (persistent attention), dense collect
# tests, the int8-scan phase stamps, and the configs[2] rerank step A/B (armi GEMM / persistent
# attention vs hipBLASLt + GELU pass / one-shot attention).
TAG=${1:-r03c}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
j() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($2)"; }
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gemm_gpu.py tests/test_encoder_gpu.py tests/test_dense_collect_gpu.py \
  tests/test_dense_filter_gpu.py > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/probes/gemm_bench.py > gpurun_out/${TAG}_gemm.log 2>&1 || exit $?
cat gpurun_out/${TAG}_gemm.log
ARMI_GEMM_BARRIERS=2 timeout -k 10 300 python tools/probes/gemm_bench.py > gpurun_out/${TAG}_gemm_b2.log 2>&1 || exit $?
echo "barriers=2:"; cat gpurun_out/${TAG}_gemm_b2.log
RR="--workload hybrid_rerank --steps 4 --warmup 2 --latency-iters 1 --no-cpu-baseline"
timeout -k 10 400 python bench.py $RR > gpurun_out/${TAG}_rerank.log 2>&1 || exit $?
echo "rerank armi: $(j gpurun_out/${TAG}_rerank.log 'round(d["value"],1), round(d["roofline"]["avg_forward_ms"],2), round(d["roofline"]["frac"],3), round(d["roofline_scan"]["avg_launch_ms"],4), d["roofline_scan"]["kernel"]')"
ARMI_RERANK_GEMM=torch ARMI_ATTENTION=oneshot timeout -k 10 400 python bench.py $RR > gpurun_out/${TAG}_rerank_old.log 2>&1 || exit $?
echo "rerank old: $(j gpurun_out/${TAG}_rerank_old.log 'round(d["value"],1), round(d["roofline"]["avg_forward_ms"],2), round(d["roofline"]["frac"],3)')"
bash tools/probes/i8_stamps.sh ${TAG}stp
