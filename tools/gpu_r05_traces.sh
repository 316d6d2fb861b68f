#!/bin/bash
# Kernel-trace summaries (rocprofv3 --kernel-trace --stats) of the bench lines the round-5 notes
# quote: the dense headline (1M), configs[1] (100k), 10k, hybrid (configs[2] retrieval) and
# hybrid_rerank. Each run under its own limit; the first failure ends the session.
TAG=${1:-r05m}
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out/$TAG"
run() {  # name, limit, bench args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$TAG/$name" -o run -- \
    python3 "$R/bench.py" "$@" > "$R/gpurun_out/$TAG/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
Q="--no-cpu-baseline --no-extras --latency-iters 3"
run dense 300 --steps 50 --warmup 5 $Q || exit $?
run c1 300 --chunks 100000 --steps 200 --warmup 10 $Q || exit $?
run c10k 300 --chunks 10000 --steps 200 --warmup 10 $Q || exit $?
run hybrid 300 --workload hybrid --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 3 || exit $?
run rerank 400 --workload hybrid_rerank --steps 3 --warmup 1 --latency-iters 1 --no-cpu-baseline || exit $?
exit 0
