#!/bin/bash
# TunableOp probe: tune the cross-encoder GEMM shapes of the hybrid_rerank bench (rocBLAS +
# hipBLASLt solutions timed per shape), then re-run the bench reading the tuned table only.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
export PYTORCH_TUNABLEOP_FILENAME="$R/gpurun_out/tunableop_results%d.csv"
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=60 \
  timeout -k 10 700 python -u bench.py --workload hybrid_rerank --steps 2 --warmup 1 --latency-iters 1 --no-cpu-baseline \
  > gpurun_out/tune_pass.log 2>&1 || exit $?
echo "tuned: $(tail -1 gpurun_out/tune_pass.log | cut -c1-300)"
timeout -k 10 300 python -u bench.py --workload hybrid_rerank --steps 5 --warmup 2 --latency-iters 3 --no-cpu-baseline \
  > gpurun_out/untuned.log 2>&1 || exit $?
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 \
  timeout -k 10 300 python -u bench.py --workload hybrid_rerank --steps 5 --warmup 2 --latency-iters 3 --no-cpu-baseline \
  > gpurun_out/tuned.log 2>&1 || exit $?
python - <<'PY'
import json
for f in ("untuned", "tuned"):
    d = json.loads(open(f"gpurun_out/{f}.log").read().strip().splitlines()[-1])
    print(f, round(d["value"], 1), "qps", d["roofline"]["avg_forward_ms"], "ms/forward", round(d["roofline"]["frac"], 3))
PY
