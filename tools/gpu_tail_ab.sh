#!/bin/bash
# (record: dense_tail_kernel and ARMI_DENSE_TAIL were removed after this A/B, profiles/r06_dense_tail_ab.txt)
# Dense tail A/B: ARMI_DENSE_TAIL=1 (merge + collect pass + collect merge in one launch) vs 0
# (three launches), interleaved, 1M and 100k rows; then the dense parity tests under the default.
TAG=${1:-tail}
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 1
out="gpurun_out/${TAG}_tail_ab.txt"
: > "$out"
for rep in 1 2; do
  for v in 1 0; do
    for n in 1000000 100000; do
      ARMI_DENSE_TAIL=$v timeout -k 10 240 python bench.py --chunks $n --steps 200 --warmup 20 --no-cpu-baseline --no-extras --latency-iters 2 > gpurun_out/${TAG}_b.json 2>/dev/null || exit $?
      python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/${TAG}_b.json') if l.startswith('{')][-1])
print('tail=$v', $n, round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))" >> "$out"
    done
  done
done
cat "$out"
