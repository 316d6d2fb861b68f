#!/bin/bash
# The driver's default bench line (dense headline + configs1 / configs2 / 10k / 10M children), timed.
TAG=${1:-r03w}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
T0=$(date +%s)
timeout -k 10 900 python bench.py > gpurun_out/${TAG}_bench_dense.log 2>&1; rc=$?
echo "rc=$rc secs=$(( $(date +%s) - T0 ))"
[ $rc -eq 0 ] || exit $rc
tail -1 gpurun_out/${TAG}_bench_dense.log | python -c "
import json, sys
d = json.loads(sys.stdin.read())
print('dense', round(d['value']), round(d['ms_per_step'], 4), round(d['roofline']['frac'], 3))
for k in ('configs1', 'configs2', 'chunks_10k', 'chunks_10M'):
    e = d.get(k, {})
    print(k, round(e['value'], 1) if 'value' in e else e, round(e.get('ms_per_step', 0), 4),
          round(e['roofline']['frac'], 3) if 'roofline' in e else None)
"
