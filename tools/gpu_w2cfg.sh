#!/bin/bash
# W=2 configs (N=16 trot, N=20 pace, mixed N=10) for product vs variants
set -o pipefail
out=$1; vars=$2
mkdir -p $(dirname $out)
for spec in "16 trot 65536" "20 pace 65536" "10 mixed 131072"; do
  set -- $spec
  N=$1 GAIT=$2 timeout -k 10 120 python tools/perf_kernel.py default $3 3 >> $out 2>&1 || exit 1
  for v in $vars; do
    QLOCO_LIB=tools/_var/$v/libqloco.so N=$1 GAIT=$2 timeout -k 10 120 python tools/perf_kernel.py default $3 3 >> $out 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $out
