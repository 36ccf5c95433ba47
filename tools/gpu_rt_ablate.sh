#!/bin/bash
# rt_pre ablations (timing only): steady-state kernel times per variant
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rtab
for v in prod ab_INTERP ab_FOOT ab_ROT ab_REF; do
  lib=""; [ $v != prod ] && lib=tools/_var/$v/libqloco.so
  QLOCO_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/rtab/$v -o run -- python tools/bench_rt.py --sets 10 --no-cpu-baseline --steps 30 > gpurun_out/rtab/$v.log 2>&1 || exit 1
  echo "== $v"; python tools/steady_kernels.py gpurun_out/rtab/$v | grep rt_pre
done
