#!/bin/bash
# configs[3] per-rank shape (tools/shard_bench.py): kernel trace + stats, then the two PMC passes
# of tools/gpu_pmc.sh over the tiled int8 scan. TAG=$1.
TAG=${1:-c3}
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_trace" -o run -- python3 "$R/tools/shard_bench.py" --chunks 10000000 --gs 8 --iters 10 > "$R/gpurun_out/${TAG}_trace.log" 2>&1 || exit $?
PMC_MATCH=gemm_scan bash "$R/tools/gpu_pmc.sh" "${TAG}_pmc" python3 "$R/tools/shard_bench.py" --chunks 10000000 --gs 8 --iters 5
