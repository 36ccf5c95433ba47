#!/bin/bash
# W=1 (N=10 trot) time breakdown: setup-only, fixed 150 iterations, default,
# at 1 / 3 / 4 waves per SIMD (B = 1024 / 3072 / 4096) and B = 8192.
set -o pipefail
out=${1:-gpurun_out/w1.log}
mkdir -p $(dirname $out)
for v in iter1 iter150 default; do
  for b in 1024 3072 4096 8192; do
    N=10 GAIT=trot timeout -k 10 120 python tools/perf_kernel.py $v $b 5 >> $out 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $out
