#!/bin/bash
# Int8-filter scan ablations (probe builds, results wrong): ARMI_I8_ABL=1 no int8->fp16
# conversion, 2 no MFMAs; dense bench kernel time of each vs the product build.
TAG=${1:-i8x}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
kt() { tail -1 $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["ms_per_step"],3), "scan_ms", round(2.052131e9/r["achieved"]/1e6, 4))'; }
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 2 > gpurun_out/${TAG}_prod.log 2>&1 || exit $?
echo "product: $(kt gpurun_out/${TAG}_prod.log)"
for a in 1 2; do
  ARMI_BUILD_FLAGS="-DARMI_PROBE_BUILD -DARMI_I8_ABL=$a" timeout -k 10 300 python -c "from audio_rag_amd import build; build.build()" > gpurun_out/${TAG}_build$a.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 2 > gpurun_out/${TAG}_abl$a.log 2>&1 || exit $?
  echo "ablate $a: $(kt gpurun_out/${TAG}_abl$a.log)"
done
