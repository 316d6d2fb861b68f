#!/bin/bash
# Round-6 final-tree evidence, part 1: the -m gpu suite, smoke, then the kernel traces of the
# bench lines the notes quote (tools/gpu_r05_traces.sh: dense 1M, configs[1], 10k, hybrid,
# hybrid_rerank). The default bench line is a separate call (tools/gpu_r06.sh). Each GPU step
# under its own limit; the first failure ends the session.
TAG=${1:-r06f}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="gpurun_out/$TAG"; mkdir -p "$O"
(while true; do date >> "$O/heartbeat.txt"; sleep 50; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { echo "$(date +%T) $1"; }
step pytest
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1; rc=$?
tail -3 "$O/pytest.log"
[ $rc -eq 0 ] || exit $rc
step smoke
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit $?
step traces
bash tools/gpu_r05_traces.sh "$TAG" || exit $?
step done
