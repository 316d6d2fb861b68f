#!/bin/bash
# dense int8 scan A/B: parity of each build, interleaved bench 1M / 100k lines, stamps
# (default build vs the ARMI_BUILD_FLAGS variants under ablibs/, e.g. VARIANTS="sortdpp")
TAG=${1:-img}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
V=${VARIANTS:-"sortdpp"}
for v in default $V; do
  L=""; [ $v != default ] && L=$PWD/ablibs/$v/libarmi.so
  ARMI_LIB_PATH=$L timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_dense_gpu.py tests/test_dense_filter_gpu.py tests/test_shards_gpu.py tests/test_sparse_rrf_gpu.py > gpurun_out/${TAG}_pytest_$v.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/${TAG}_pytest_$v.log)"
done
for rep in 1 2; do
  for v in default $V; do
    L=""; [ $v != default ] && L=$PWD/ablibs/$v/libarmi.so
    for n in 1000000 100000; do
      ARMI_LIB_PATH=$L timeout -k 10 120 python bench.py --steps 300 --warmup 30 --chunks $n --no-cpu-baseline --no-extras > gpurun_out/${TAG}_${v}_${n}_$rep.json 2> gpurun_out/${TAG}_${v}_${n}_$rep.err || exit 1
      python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],sys.argv[3],round(d['value']),round(d['ms_per_step'],4),round(d['roofline']['avg_launch_ms'],4))" gpurun_out/${TAG}_${v}_${n}_$rep.json $v $n
    done
  done
done
for s in ${STAMPS:-stamps}; do
  [ -f ablibs/$s/libarmi.so ] || continue
  for n in 1000000 100000; do
    ARMI_LIB_PATH=$PWD/ablibs/$s/libarmi.so timeout -k 10 200 python tools/probes/i8_stamps.py --chunks $n > gpurun_out/${TAG}_${s}_$n.log 2>&1 || exit 1
    tail -1 gpurun_out/${TAG}_${s}_$n.log | python -c "import json,sys;d=json.loads(sys.stdin.read());m=d['median_us'];print(sys.argv[1],{k:round(v,1) for k,v in m.items() if not k.startswith('xcd')})" $s
  done
done
# hybrid (configs[2] retrieval) lines: default vs HYB_VARIANTS
if [ -n "$HYB_VARIANTS" ]; then
  for rep in 1 2; do
    for v in default $HYB_VARIANTS; do
      L=""; [ $v != default ] && L=$PWD/ablibs/$v/libarmi.so
      ARMI_LIB_PATH=$L timeout -k 10 180 python bench.py --workload hybrid --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/${TAG}_hyb_${v}_$rep.json 2> gpurun_out/${TAG}_hyb_${v}_$rep.err || exit 1
      python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline_sparse') or {};print('hybrid',sys.argv[2],round(d['value']),round(d['ms_per_step'],4),round(r.get('avg_launch_ms',0),4))" gpurun_out/${TAG}_hyb_${v}_$rep.json $v
    done
  done
fi
