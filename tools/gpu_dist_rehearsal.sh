#!/bin/bash
# Rehearsal of bench.py's N>1 path on a one-GPU box: N ranks share cuda:0 and exchange over gloo
# (RCCL refuses two ranks on one device). Exercises the real kernels, the all-gathers of queries
# and per-shard top-k, armi_topk_merge_shards and RRF after the merge; the timing is not a
# scaling number (the ranks share one GPU).
TAG=${1:-r02g}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
export ARMI_BENCH_BACKEND=gloo
for n in 2 4; do
  for wl in dense hybrid; do
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 2 \
      --latency-iters 2 --workload $wl > gpurun_out/${TAG}_dist_${wl}_n$n.log 2>&1 || exit $?
    echo "n=$n $wl: $(tail -1 gpurun_out/${TAG}_dist_${wl}_n$n.log | cut -c1-160)"
  done
done
