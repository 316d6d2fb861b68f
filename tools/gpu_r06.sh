#!/bin/bash
# Round-6 GPU session: tag=$1; TESTS = pytest targets (default: the whole -m gpu suite);
# BENCH=0 skips the default bench line. Every GPU step has its own time limit and a crash-like
# exit ends the session; a heartbeat file under gpurun_out/ marks progress of long steps.
TAG=${1:-r06}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
(while true; do date >> gpurun_out/${TAG}_heartbeat.txt; sleep 50; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test failures (no crash)
if [ "${TESTS:-none}" != "none" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS} -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"
  tail -3 gpurun_out/${TAG}_pytest.log
  ok $rc || exit $rc
fi
if [ "${SMOKE:-0}" = "1" ]; then
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"
  ok $rc || exit $rc
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-1000} python -u bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err; rc=$?; echo "bench rc=$rc"
  tail -c 600 gpurun_out/${TAG}_bench.json
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${EXTRA}" ]; then
  bash -c "${EXTRA}"; rc=$?; echo "extra rc=$rc"; exit $rc
fi
exit 0
