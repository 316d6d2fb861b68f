#!/bin/bash
# GPU test session: the given pytest selection (default: every -m gpu test), one process, each
# step under its own limit; stops at the first step that fails abnormally.
TAG=${1:-t}; shift
SEL=${*:-tests}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $SEL -m gpu -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|certified|error =|cos " gpurun_out/${TAG}_pytest.log | tail -40
exit $rc
