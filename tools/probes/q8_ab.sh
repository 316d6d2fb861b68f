#!/bin/bash
# Int8-query form of the filter scan (k <= 6): GPU suite, then dense bench with int8 queries
# (default) vs fp16 queries (ARMI_DENSE_QUERY=fp16) vs the fp16 scan (ARMI_DENSE_FILTER=fp16).
TAG=${1:-q8}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
run() {
  timeout -k 10 400 env $2 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 10 > gpurun_out/${TAG}_$1.log 2>&1 || exit $?
  echo "$1: $(tail -1 gpurun_out/${TAG}_$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]), round(d["ms_per_step"],3), "p50", round(d["p50_ms"],3), "scan_ms", round(r["avg_launch_ms"],4), round(r["frac"],3), "cert", d["certified_frac"])')"
}
run q8 ARMI_X=0
run f16q ARMI_DENSE_QUERY=fp16
run fp16 ARMI_DENSE_FILTER=fp16
run q8b ARMI_X=0
