#!/bin/bash
# GPU session: tag=$1. Each GPU step has its own time limit; a crash-like exit ends the session.
TAG=${1:-run}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test failures (no crash)
timeout -k 10 600 python -m pytest tests -v -m "${MARK:-gpu}" > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"
ok $rc || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"
ok $rc || exit $rc
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.log 2>&1; rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
[ -n "${NO_PROF}" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" 2>&1; rc=$?; echo "prof rc=$rc"
exit $rc
