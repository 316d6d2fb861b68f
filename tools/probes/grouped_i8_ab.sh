#!/bin/bash
# Per-rank compute of the sharded dense step (tools/shard_bench.py): tiled four-wave scan (fp16)
# vs the XCD-grouped 64-query int8 filter scan forced for > 128 queries (ARMI_DENSE_SCAN=grouped).
TAG=${1:-gi8}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
for f in tiled grouped tiled grouped; do
  ARMI_DENSE_SCAN=$f timeout -k 10 300 python tools/shard_bench.py --gs 1,2,4,8 > gpurun_out/${TAG}_$f.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/${TAG}_$f.log | sed "s/^/$f: /"
done
ARMI_DENSE_SCAN=grouped timeout -k 10 300 python tools/shard_bench.py --gs 8 --chunks 10000000 > gpurun_out/${TAG}_g10m.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/${TAG}_g10m.log | sed "s/^/grouped 10M: /"
