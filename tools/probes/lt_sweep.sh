#!/bin/bash
# hipBLASLt solution sweeps: the Q x C scan shapes (fp16 and fp32 output) at 1.25M rows, then the
# cross-encoder projections at 327,680 rows, all on random operands.
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 240 ./tools/probes/lt_sweep 1250000 4 600 scan h > gpurun_out/lt_scan_h.txt 2>&1 || exit $?
timeout -k 10 240 ./tools/probes/lt_sweep 1250000 4 600 scan f > gpurun_out/lt_scan_f.txt 2>&1 || exit $?
timeout -k 10 300 ./tools/probes/lt_sweep 327680 4 600 enc h > gpurun_out/lt_enc_h.txt 2>&1 || exit $?
for f in lt_scan_h lt_scan_f lt_enc_h; do echo "== $f"; grep -v "^  idx" gpurun_out/$f.txt | cut -c1-90; grep "^  idx" gpurun_out/$f.txt | cut -c1-60; done
