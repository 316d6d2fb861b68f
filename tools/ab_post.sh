#!/bin/bash
# A/B of two libarmi builds on one box: tools/ab_post.sh OUT LIB_B [bench args]; A = the in-tree lib
OUT=$1; LIBB=$2; shift 2
mkdir -p "$OUT"
for rep in 1 2; do
  for v in A B; do
    if [ $v = B ]; then export ARMI_LIB_PATH=$LIBB; else unset ARMI_LIB_PATH; fi
    for ch in 1000000 100000 10000; do
      timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-extras --chunks $ch --latency-iters 3 "$@" > "$OUT/${v}_${ch}_${rep}.json" 2> "$OUT/${v}_${ch}_${rep}.err" || exit 1
    done
  done
done
