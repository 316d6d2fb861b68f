#!/bin/bash
# dense_scan_i8_kernel phase timeline (probe build with s_memrealtime stamps; results unchanged)
TAG=${1:-stp}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
ARMI_BUILD_FLAGS="-DARMI_PROBE_BUILD -DARMI_I8_STAMPS" timeout -k 10 300 python -c "from audio_rag_amd import build; build.build()" > gpurun_out/${TAG}_build.log 2>&1 || exit $?
for n in 100000 1000000 4000000; do
  timeout -k 10 200 python tools/probes/i8_stamps.py --chunks $n > gpurun_out/${TAG}_$n.log 2>&1 || exit $?
  tail -1 gpurun_out/${TAG}_$n.log
done
