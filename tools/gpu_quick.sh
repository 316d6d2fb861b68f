#!/bin/bash
# quick GPU check: selected tests + one bench workload
TAG=${1:-q}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest ${TESTS:-tests} -v -m "gpu and not slow" > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.log 2>&1; rc=$?; echo "bench rc=$rc"
exit $rc
