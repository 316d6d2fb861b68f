#!/bin/bash
# PMC traffic of the int8 scan (first pass only) + phase stamps with per-workgroup spreads.
TAG=${1:-r03h}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
bash tools/gpu_pmc_i8.sh ${TAG}pmc || exit $?
cd "$R" && bash tools/probes/i8_stamps.sh ${TAG}stp || exit $?
