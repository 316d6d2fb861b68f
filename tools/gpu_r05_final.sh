#!/bin/bash
# Round-5 final-tree evidence: the -m gpu suite, smoke, the default bench line (with its child
# configs), the hybrid / hybrid_rerank / pipeline / stream lines, then the kernel traces of
# tools/gpu_r05_traces.sh. Each GPU step under its own limit; the first failure ends the session.
TAG=${1:-r05z}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="gpurun_out/$TAG"; mkdir -p "$O"
step() { echo "$(date +%T) $1"; }
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || exit $?
step smoke
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit $?
step bench_default
timeout -k 10 400 python -u bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || exit $?
step bench_hybrid
timeout -k 10 200 python -u bench.py --workload hybrid --no-cpu-baseline --no-extras > "$O/bench_hybrid.json" 2> "$O/bench_hybrid.err" || exit $?
step bench_pipeline
timeout -k 10 300 python -u bench.py --workload pipeline --no-cpu-baseline --no-extras > "$O/bench_pipeline.json" 2> "$O/bench_pipeline.err" || exit $?
step bench_stream
timeout -k 10 300 python -u bench.py --workload stream --no-cpu-baseline --no-extras > "$O/bench_stream.json" 2> "$O/bench_stream.err" || exit $?
step traces
bash tools/gpu_r05_traces.sh "$TAG" || exit $?
step done
