#!/bin/bash
# A/B of two libarmi builds on one box over bench.py shard sizes:
# tools/ab_libs.sh OUT LIB_B "CHUNKS..." [bench args]; A = the in-tree lib, two rounds each
OUT=$1; LIBB=$2; CHUNKS=$3; shift 3
mkdir -p "$OUT"
for rep in 1 2; do
  for v in A B; do
    if [ $v = B ]; then export ARMI_LIB_PATH=$LIBB; else unset ARMI_LIB_PATH; fi
    for ch in $CHUNKS; do
      timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-extras --chunks $ch --latency-iters 3 "$@" > "$OUT/${v}_${ch}_${rep}.json" 2> "$OUT/${v}_${ch}_${rep}.err" || exit 1
    done
  done
done
for f in "$OUT"/*.json; do
  python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step'], 4), round(d['value']))"
done
