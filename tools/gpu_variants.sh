#!/bin/bash
# time experimental builds (tools/_var/NAME/libqloco.so) against the product library
# usage: bash tools/gpu_variants.sh OUT "VAR1 VAR2 ..." "B1 B2 ..." [N] [GAIT]
set -o pipefail
out=$1; vars=$2; bs=$3; n=${4:-10}; gait=${5:-trot}
mkdir -p $(dirname $out)
for b in $bs; do
  N=$n GAIT=$gait timeout -k 10 120 python tools/perf_kernel.py default $b 5 >> $out 2>&1 || exit 1
  for v in $vars; do
    QLOCO_LIB=tools/_var/$v/libqloco.so N=$n GAIT=$gait timeout -k 10 120 python tools/perf_kernel.py default $b 5 >> $out 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $out
