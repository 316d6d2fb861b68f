#!/bin/bash
# Dense int8 first pass: static ranges vs a dynamic tail (ARMI_I8_TAIL_STATIC builds under ablibs/).
# Record of the r04ah A/B (profiles/r04ah_dense_tail_ab.txt): the tail form and its build flag were removed after it.
# Parity of each variant under -m gpu, then interleaved 1M / 100k bench lines and the stamps.
TAG=${1:-tab}
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
V=${VARIANTS:-"tail875 tail750"}
for v in $V; do
  ARMI_LIB_PATH=$PWD/ablibs/$v/libarmi.so timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_dense_gpu.py tests/test_dense_filter_gpu.py > gpurun_out/${TAG}_pytest_$v.log 2>&1 || { tail -20 gpurun_out/${TAG}_pytest_$v.log; exit 1; }
  tail -1 gpurun_out/${TAG}_pytest_$v.log
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
if [ -f ablibs/stamps_tail/libarmi.so ]; then
  ARMI_LIB_PATH=$PWD/ablibs/stamps_tail/libarmi.so timeout -k 10 200 python tools/probes/i8_stamps.py --chunks 1000000 > gpurun_out/${TAG}_stamps_tail.log 2>&1 && tail -1 gpurun_out/${TAG}_stamps_tail.log
  ARMI_LIB_PATH=$PWD/ablibs/stamps/libarmi.so timeout -k 10 200 python tools/probes/i8_stamps.py --chunks 1000000 > gpurun_out/${TAG}_stamps_static.log 2>&1 && tail -1 gpurun_out/${TAG}_stamps_static.log
fi
