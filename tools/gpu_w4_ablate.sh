#!/bin/bash
# Timing-only ablations of the tiled int8 scan at the configs[3] per-rank shape: probe builds
# (ARMI_BUILD_FLAGS="-DARMI_PROBE_BUILD -DARMI_W4_ABL=a", results wrong) against the in-tree build.
cd "$GRAFT_REPO_ROOT" || exit 1
for v in tree 1 2 4 8; do
  if [ $v = tree ]; then unset ARMI_AB_OTHER_SOURCES ARMI_LIB_PATH; else export ARMI_AB_OTHER_SOURCES=1 ARMI_LIB_PATH=audio_rag_amd/_lib/probe/libarmi_abl$v.so; fi
  echo "== $v" >> gpurun_out/w4abl.log
  timeout -k 10 300 python tools/shard_bench.py --chunks 10000000 --gs 8 --iters 10 >> gpurun_out/w4abl.log 2>&1 || exit $?
done
cat gpurun_out/w4abl.log
