#!/bin/bash
# Int8-filter 64-query scan: dense / fullsize / store / batcher parity, then the dense bench line
# with the int8 pass (default) and with the fp16 scan (ARMI_DENSE_FILTER=fp16).
TAG=${1:-i8}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
for f in i8 fp16 i8; do
  if [ $f = fp16 ]; then export ARMI_DENSE_FILTER=fp16; else unset ARMI_DENSE_FILTER; fi
  timeout -k 10 400 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_$f.log 2>&1 || exit $?
  echo "$f: $(tail -1 gpurun_out/${TAG}_bench_$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],3), d["p50_ms"] if "p50_ms" in d else "", d["roofline"]["achieved"], round(d["roofline"]["frac"],3), d.get("certified"))')"
done
unset ARMI_DENSE_FILTER
timeout -k 10 400 python bench.py --workload hybrid --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench_hybrid.log 2>&1 || exit $?
echo "hybrid: $(tail -1 gpurun_out/${TAG}_bench_hybrid.log | cut -c1-200)"
