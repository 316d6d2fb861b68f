#!/bin/bash
# A/B of the in-tree library against a probe build (ARMI_LIB_PATH=$1) on one command ($2...),
# interleaved, two reps; outputs under gpurun_out/libab_*.log
B="$1"; shift
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export ARMI_AB_OTHER_SOURCES=1 ARMI_LIB_PATH="$B"; else unset ARMI_AB_OTHER_SOURCES ARMI_LIB_PATH; fi
    echo "== $v rep $rep" >> gpurun_out/libab.log
    timeout -k 10 300 "$@" >> gpurun_out/libab.log 2>&1 || exit $?
  done
done
cat gpurun_out/libab.log
