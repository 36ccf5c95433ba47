#!/bin/bash
# Reduced two-wave C2 = 15 bucket: three waves per SIMD (shipped, 33 spilled
# VGPRs outside the ADMM loop) vs two (tools/_var/c15w2: the warm
# instantiation's budget, spill-free), configs-3 / 4 shapes, alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r6ai; mkdir -p $out
for k in 1 2; do
  for v in prod c15w2; do
    if [ $v = prod ]; then unset QLOCO_LIB; else export QLOCO_LIB=$PWD/tools/_var/c15w2/libqloco.so; fi
    N=16 GAIT=trot timeout -k 10 120 python tools/perf_kernel.py default 65536 10 >> $out/ab.txt 2>> $out/err.txt || { tail $out/err.txt; exit 1; }
    N=20 GAIT=pace timeout -k 10 120 python tools/perf_kernel.py default 65536 10 >> $out/ab.txt 2>> $out/err.txt || { tail $out/err.txt; exit 1; }
    N=10 GAIT=mixed timeout -k 10 120 python tools/perf_kernel.py default 131072 10 >> $out/ab.txt 2>> $out/err.txt || { tail $out/err.txt; exit 1; }
  done
done
cat $out/ab.txt
