#!/bin/bash
# C2 = 6 two-wave bucket at four waves/SIMD for N <= 10 (tools/_var/c6w4,
# -DQLOCO_SRBD_W2_C6_SHORT_WPE=4) vs the shipped three-wave instantiation on
# the mixed config-5 share, and the bench step's timing-event overhead.
# Usage: tools/gpu_r3_c6.sh TAG
set -o pipefail
tag=${1:-r3c6}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python tools/event_overhead.py 4096 200 > $out/events.txt 2>&1 || { tail -5 $out/events.txt; exit 1; }
grep -v amdgpu.ids $out/events.txt
for rep in 1 2; do
  for L in "" tools/_var/c6w4/libqloco.so; do
    GAIT=mixed N=10 QLOCO_LIB=$L timeout -k 10 180 python tools/perf_kernel.py default 131072 5 >> $out/ab.txt 2>&1 || { tail -5 $out/ab.txt; exit 1; }
  done
done
grep -v amdgpu.ids $out/ab.txt
