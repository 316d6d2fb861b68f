#!/bin/bash
# Int8 scan load policy: default vs non-temporal (probe build -DARMI_I8_NT), dense bench.
TAG=${1:-nt}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
kt() { tail -1 $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]), round(d["ms_per_step"],3), "scan_ms", round(r["avg_launch_ms"],4))'; }
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 2 > gpurun_out/${TAG}_def.log 2>&1 || exit $?
echo "default: $(kt gpurun_out/${TAG}_def.log)"
ARMI_BUILD_FLAGS="-DARMI_PROBE_BUILD -DARMI_I8_NT" timeout -k 10 300 python -c "from audio_rag_amd import build; build.build()" > gpurun_out/${TAG}_build.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 2 > gpurun_out/${TAG}_nt.log 2>&1 || exit $?
echo "nt: $(kt gpurun_out/${TAG}_nt.log)"
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 2 > gpurun_out/${TAG}_nt2.log 2>&1 || exit $?
echo "nt: $(kt gpurun_out/${TAG}_nt2.log)"
