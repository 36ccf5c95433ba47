#!/bin/bash
# BASELINE configs 2-5 on one GPU (per-GPU shares for the 8-GPU configs)
set -o pipefail
out=${1:-gpurun_out/configs.log}
mkdir -p $(dirname $out)
for spec in "10 trot 4096" "16 trot 65536" "20 pace 65536" "10 mixed 131072" "10 pace 4096" "10 mixed 4096"; do
  set -- $spec
  N=$1 GAIT=$2 timeout -k 10 120 python tools/perf_kernel.py default $3 5 >> $out 2>&1 || exit 1
done
grep -v amdgpu.ids $out
