#!/bin/bash
for n in 1000000 100000 10000; do python bench.py --chunks $n --steps 200 --warmup 20 --no-cpu-baseline --no-extras --latency-iters 2 2>/dev/null | python3 -c "
import json,sys
d=json.loads([l for l in sys.stdin if l.startswith('{')][-1])
print($n, round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"; done
