#!/bin/bash
# Round-4 GPU session: full -m gpu suite + smoke, the default bench line (driver shape, with the
# configs1 / configs2 children and their CPU baselines), the single-query search breakdown,
# rocprofv3 kernel stats of the dense bench and the per-shape PMC traffic passes.
# Each GPU step has its own limit; any failure ends the session.
TAG=${1:-r04a}
STEPS=${2:-all}
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 1
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
if [[ $STEPS == all || $STEPS == *tests* ]]; then
  timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc: $(tail -1 gpurun_out/${TAG}_pytest.log)"
  grep -E "FAILED|ERROR" gpurun_out/${TAG}_pytest.log | head -20
  ok $rc || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
  echo "smoke: $(tail -1 gpurun_out/${TAG}_smoke.log)"
fi
if [[ $STEPS == all || $STEPS == *bench* ]]; then
  t0=$(date +%s)
  timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
  echo "bench wall $(( $(date +%s) - t0 )) s"
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print('dense',round(d['value']),'ms',round(d['ms_per_step'],4),'frac',round(d['roofline']['frac'],3),'traffic',d['roofline']['traffic'],'cpu',d['cpu_baseline']['value']);[print(k,round(d[k].get('value',0)),d[k].get('cpu_baseline',{}) and d[k]['cpu_baseline']['value'],d[k].get('roofline',{}).get('traffic')) for k in ('configs1','configs2','chunks_10k','chunks_10M')]"
fi
if [[ $STEPS == all || $STEPS == *lat* ]]; then
  timeout -k 10 300 python tools/search_latency.py > gpurun_out/${TAG}_search_latency.json 2>&1 || exit $?
  cat gpurun_out/${TAG}_search_latency.json
fi
if [[ $STEPS == all || $STEPS == *prof* ]]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_prof_dense" -o run -- \
    python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-extras --latency-iters 3 > "$R/gpurun_out/${TAG}_prof_dense.log" 2>&1 || exit $?
  echo "prof dense done"
  cd "$R"
fi
if [[ $STEPS == all || $STEPS == *pmc1m* ]]; then
  bash tools/pmc_traffic.sh ${TAG}_t1m roofline || exit $?
fi
if [[ $STEPS == all || $STEPS == *pmc100k* ]]; then
  bash tools/pmc_traffic.sh ${TAG}_t100k roofline --chunks 100000 || exit $?
  bash tools/pmc_traffic.sh ${TAG}_t10k roofline --chunks 10000 || exit $?
fi
if [[ $STEPS == all || $STEPS == *pmcsp* ]]; then
  bash tools/pmc_traffic.sh ${TAG}_tsp roofline_sparse --workload hybrid || exit $?
fi
if [[ $STEPS == *sqsparse* ]]; then
  bash tools/probes/pmc_sparse.sh ${TAG}_sqsp || exit $?
fi
if [[ $STEPS == *rerankprof* ]]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_prof_rerank" -o run -- \
    python3 "$R/bench.py" --workload hybrid_rerank --steps 3 --warmup 2 --latency-iters 1 --no-cpu-baseline > "$R/gpurun_out/${TAG}_prof_rerank.log" 2>&1 || exit $?
  echo "prof rerank done"; tail -1 "$R/gpurun_out/${TAG}_prof_rerank.log" | cut -c1-300
  cd "$R"
fi
if [[ $STEPS == *hybrid* ]]; then
  timeout -k 10 300 python bench.py --workload hybrid --no-cpu-baseline --steps 40 --warmup 5 --latency-iters 5 > gpurun_out/${TAG}_bench_hybrid.json 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_bench_hybrid.json').read().strip().splitlines()[-1]);r=d['roofline_sparse'];print('hybrid',round(d['value']),'ms',round(d['ms_per_step'],4),'sparse scan ms',round(r['avg_launch_ms'],4),'frac',round(r['frac'],3))"
fi
if [[ $STEPS == *gemm* ]]; then
  timeout -k 10 300 python tools/probes/gemm_bench.py > gpurun_out/${TAG}_gemm.log 2>&1 || exit $?
  grep '^{' gpurun_out/${TAG}_gemm.log
fi
if [[ $STEPS == *pipeline* ]]; then
  timeout -k 10 500 python bench.py --workload pipeline --queries 200 > gpurun_out/${TAG}_bench_pipeline.json 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_bench_pipeline.json').read().strip().splitlines()[-1]);print('pipeline p50',d['p50_ms'],d['stage_p50_ms'])"
fi
exit 0
