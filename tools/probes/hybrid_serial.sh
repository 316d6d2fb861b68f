cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for m in conc serial conc serial; do
  if [ $m = serial ]; then export ARMI_HYBRID_SERIAL=1; else unset ARMI_HYBRID_SERIAL; fi
  timeout -k 10 300 python bench.py --workload hybrid --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 2 > gpurun_out/hs_$m.log 2>&1 || exit 1
  echo "$m $(tail -1 gpurun_out/hs_$m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],4))')"
done
