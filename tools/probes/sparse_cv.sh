#!/bin/bash
# Sparse compute-loop variants (ARMI_SPARSE_CV builds libarmi_cv<N>.so): sparse_bench time each.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; mkdir -p gpurun_out
L=audio_rag_amd/_lib
cp $L/libarmi.so $L/libarmi_norm.so
for v in "$@"; do
  cp $L/libarmi_cv$v.so $L/libarmi.so
  for r in 1 2; do
    timeout -k 10 300 python tools/sparse_bench.py --iters 100 > gpurun_out/cv${v}_$r.log 2>&1 || { cp $L/libarmi_norm.so $L/libarmi.so; exit 1; }
    echo "cv$v: $(tail -1 gpurun_out/cv${v}_$r.log)"
  done
done
cp $L/libarmi_norm.so $L/libarmi.so
