#!/bin/bash
# Round-2 check-in session: full -m gpu suite, smoke, dense bench, kernel-trace stats of the dense
# bench. Each GPU step has its own limit; a crash / timeout ends the session.
TAG=${1:-r02a}
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 1
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc: $(tail -1 gpurun_out/${TAG}_pytest.log)"
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
echo "smoke: $(tail -1 gpurun_out/${TAG}_smoke.log)"
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench_dense.log 2>&1 || exit $?
echo "dense: $(tail -1 gpurun_out/${TAG}_bench_dense.log | cut -c1-300)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_prof_dense" -o run -- \
  python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --latency-iters 3 > "$R/gpurun_out/${TAG}_prof_dense.log" 2>&1 || exit $?
echo "prof dense done"
exit 0
