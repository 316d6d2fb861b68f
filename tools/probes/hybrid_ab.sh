#!/bin/bash
# A/B of the hybrid step on one box: the in-tree library (A) against another build (B, loaded with
# ARMI_LIB_PATH + ARMI_AB_OTHER_SOURCES=1), graphed hybrid bench, alternating, N rounds.
# tools/probes/hybrid_ab.sh OUT LIB_B [rounds]
OUT=$1; LIBB=$2; N=${3:-3}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p "$OUT"
for rep in $(seq 1 $N); do
  for v in A B; do
    if [ $v = B ]; then export ARMI_LIB_PATH=$LIBB ARMI_AB_OTHER_SOURCES=1; else unset ARMI_LIB_PATH ARMI_AB_OTHER_SOURCES; fi
    timeout -k 10 200 python -u bench.py --workload hybrid --no-cpu-baseline --no-extras > "$OUT/${v}_${rep}.json" 2> "$OUT/${v}_${rep}.err" || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/${v}_${rep}.json').read().strip().splitlines()[-1]); print('$v $rep', round(d['value']), round(d['ms_per_step'], 4))"
  done
done
