#!/bin/bash
# Kernel-timing cost A/B: bench.py with the live scan timing at periods 8 (default), 1 and 0
# (off), interleaved, 1M and 100k rows; prints q/s, ms per step, the timed scan's ms and count.
cd "$GRAFT_REPO_ROOT" || exit 1
: > gpurun_out/ev_ab.txt
for rep in 1 2; do for v in 8 1 0; do for n in 1000000 100000; do
  ARMI_BENCH_TIMING=$v timeout -k 10 240 python bench.py --chunks $n --steps 200 --warmup 20 --no-cpu-baseline --no-extras --latency-iters 2 > gpurun_out/ev_b.json 2>/dev/null || exit $?
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/ev_b.json') if l.startswith('{')][-1])
print('period=$v', $n, round(d['value']), round(d['ms_per_step'],4), d['roofline'].get('avg_launch_ms'), d['roofline'].get('launches_timed'))" >> gpurun_out/ev_ab.txt
done; done; done
cat gpurun_out/ev_ab.txt
