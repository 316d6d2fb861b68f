#!/bin/bash
# A/B of linear_f16_kernel probe builds (ablibs/libarmi_v*.so, ARMI_BUILD_FLAGS=-DARMI_GEMM_V=n)
# against the default build, alternating processes on one box: gemm_bench.py per build, twice.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
TAG=${1:-gab}; shift
export GEMM_NO_LT=1
for round in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then lib=""; else lib="$R/ablibs/libarmi_$v.so"; fi
    ARMI_LIB_PATH=$lib timeout -k 10 120 python3 tools/probes/gemm_bench.py > gpurun_out/${TAG}_${v}_$round.log 2>&1 || exit $?
    python3 -c "import json,sys;[print('$v',$round,d['shape'],round(d['armi_ms'],4),round(d['armi_tflops'])) for d in map(json.loads,[l for l in open('gpurun_out/${TAG}_${v}_$round.log') if l.startswith('{')])]"
  done
done
