#!/bin/bash
# marginal cost of setup phases at B=8192 (iter1: setup + 1 iteration):
# Ruiz passes (scaling 0/10/20), a second gen_p_row, two more inverses
set -o pipefail
out=${1:-gpurun_out/ablate.log}
mkdir -p $(dirname $out)
for v in iter1 iter1s0 iter1s20; do
  timeout -k 10 120 python tools/perf_kernel.py $v 8192 5 >> $out 2>&1 || exit 1
done
for lib in dupg dupi; do
  QLOCO_LIB=tools/_var/$lib/libqloco.so timeout -k 10 120 python tools/perf_kernel.py iter1 8192 5 >> $out 2>&1 || exit 1
done
grep -v amdgpu.ids $out
