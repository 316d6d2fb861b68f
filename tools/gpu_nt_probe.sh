#!/bin/bash
# 1M dense scan: kernel duration (rocprofv3) vs the in-kernel stamp span, nontemporal image
# stream on (default) / off (ARMI_I8_NT_MIN_MB=1e6 build), then bench A/B of the two libraries.
TAG=${1:-nt}
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
for v in i8stamps i8stamps_nont; do
  ARMI_AB_OTHER_SOURCES=1 ARMI_LIB_PATH=$R/audio_rag_amd/_lib/probe/libarmi_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_$v" -o run -- python3 "$R/tools/probes/i8_stamps.py" --chunks 1000000 > "$R/gpurun_out/${TAG}_$v.log" 2>&1 || exit $?
done
cd "$R" || exit 1
: > gpurun_out/${TAG}_ab.txt
for rep in 1 2; do for v in default nont; do
  if [ $v = default ]; then L=""; else L="ARMI_AB_OTHER_SOURCES=1 ARMI_LIB_PATH=$R/audio_rag_amd/_lib/probe/libarmi_nont.so"; fi
  env $L timeout -k 10 240 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-extras --latency-iters 2 > gpurun_out/${TAG}_b.json 2>/dev/null || exit $?
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/${TAG}_b.json') if l.startswith('{')][-1])
print('$v', round(d['value']), round(d['ms_per_step'],4), d['roofline'].get('avg_launch_ms'))" >> gpurun_out/${TAG}_ab.txt
done; done
cat gpurun_out/${TAG}_ab.txt
