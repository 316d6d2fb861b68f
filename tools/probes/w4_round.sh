#!/bin/bash
# The four-wave tiled scan as the default: full -m gpu suite, k=40 certification/time (w4 vs
# glds), rocprofv3 kernel stats and one SQ counter pass at the 10M / 8-way per-rank shape.
TAG=${1:-r02w}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || exit $rc
for f in w4 glds; do
  ARMI_GEMM_FORM=$f timeout -k 10 300 python tools/shard_bench.py --chunks 10000000 --gs 8 --k 40 > gpurun_out/${TAG}_${f}_k40.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/${TAG}_${f}_k40.log | sed "s/^/$f k40: /"
done
cd /tmp && export TMPDIR=/tmp
B="$R/tools/shard_bench.py --gs 8 --chunks 10000000 --iters 10"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof" -o run -- python3 $B > "$R/gpurun_out/${TAG}_prof.log" 2>&1 || exit $?
echo "prof: $(grep -v amdgpu.ids $R/gpurun_out/${TAG}_prof.log | tail -1)"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d "$R/gpurun_out/${TAG}_sq" -o run -- python3 $B > "$R/gpurun_out/${TAG}_sq.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TD_BUSY_avr --output-format csv -d "$R/gpurun_out/${TAG}_grbm" -o run -- python3 $B > "$R/gpurun_out/${TAG}_grbm.log" 2>&1 || exit $?
echo "pmc done"
