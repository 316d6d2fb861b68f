#!/bin/bash
# Cost of the sharded step's exchange on one GPU: bench.py's N>1 code path (query all-gather,
# packed candidate all-gather over RCCL, merge) at WORLD_SIZE 1, beside the plain N=1 step, plus a
# kernel trace of the sharded dense step (GPU busy time vs wall time per step).
TAG=${1:-r02h}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29555 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
O=gpurun_out/${TAG}_sharded_w1.txt; : > $O
for wl in dense hybrid; do
  timeout -k 10 300 python bench.py --workload $wl --steps 200 --warmup 10 --no-cpu-baseline --latency-iters 20 > gpurun_out/${TAG}_plain_$wl.log 2>&1 || exit $?
  echo "plain $wl: $(tail -1 gpurun_out/${TAG}_plain_$wl.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],4), round(d["p50_ms"],4))')" | tee -a $O
  ARMI_BENCH_SHARDED=1 timeout -k 10 300 python bench.py --workload $wl --steps 200 --warmup 10 --no-cpu-baseline --latency-iters 20 > gpurun_out/${TAG}_sharded_$wl.log 2>&1 || exit $?
  echo "sharded(world 1) $wl: $(tail -1 gpurun_out/${TAG}_sharded_$wl.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],4), round(d["p50_ms"],4))')" | tee -a $O
done
cd /tmp && export TMPDIR=/tmp ARMI_BENCH_SHARDED=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_shp -o run -- python3 $R/bench.py --steps 200 --warmup 10 --no-cpu-baseline --latency-iters 2 > $R/gpurun_out/${TAG}_shp.log 2>&1 || exit $?
python3 $R/tools/rocpd_stats.py $R/gpurun_out/${TAG}_shp/run_results.db > $R/gpurun_out/${TAG}_sharded_dense_kernel_stats.csv || exit $?
rm -rf $R/gpurun_out/${TAG}_shp
