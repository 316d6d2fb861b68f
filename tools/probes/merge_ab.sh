#!/bin/bash
# Dense parity (dense, filter, full-size dense) then the dense bench: int8 filter (default),
# int8 queries (ARMI_DENSE_QUERY=int8), fp16 scan (ARMI_DENSE_FILTER=fp16).
TAG=${1:-mg}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_dense_gpu.py tests/test_dense_filter_gpu.py tests/test_fullsize_gpu.py -k "not bge and not rerank" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
run() {
  timeout -k 10 400 env $2 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 10 > gpurun_out/${TAG}_$1.log 2>&1 || exit $?
  echo "$1: $(tail -1 gpurun_out/${TAG}_$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]), round(d["ms_per_step"],3), "p50", round(d["p50_ms"],3), "scan_ms", round(r["avg_launch_ms"],4), round(r["frac"],3), "cert", d["certified_frac"])')"
}
run i8 ARMI_X=0
run q8 ARMI_DENSE_QUERY=int8
run fp16 ARMI_DENSE_FILTER=fp16
run i8b ARMI_X=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof" -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --latency-iters 2 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" 2>&1 || exit $?
echo prof done
