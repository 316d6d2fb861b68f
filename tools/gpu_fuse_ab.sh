#!/bin/bash
# (record: the ARMI_FUSE_ON_SIDE switch was removed after this A/B, profiles/r06_rrf_stream_ab.txt)
# Hybrid step A/B: RRF on the side stream (default) vs on the caller's stream (ARMI_FUSE_ON_SIDE=0)
cd "$GRAFT_REPO_ROOT" || exit 1
: > gpurun_out/fuse_ab.txt
for rep in 1 2; do for v in 1 0; do
  ARMI_FUSE_ON_SIDE=$v timeout -k 10 300 python bench.py --workload hybrid --steps 200 --warmup 20 --no-cpu-baseline --no-extras --latency-iters 2 > gpurun_out/fuse_b.json 2>/dev/null || exit $?
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/fuse_b.json') if l.startswith('{')][-1])
print('fuse_on_side=$v', round(d['value']), round(d['ms_per_step'],4), round(d['p50_ms'],4))" >> gpurun_out/fuse_ab.txt
done; done
cat gpurun_out/fuse_ab.txt
