#!/bin/bash
# Where a configs[1] launch of the shipped four-waves/SIMD one-wave kernel
# goes (tools/perf_kernel.py variants: setup only, setup without Ruiz, 150
# check-free iterations, 150 iterations with 30 residual checks, default),
# at B = 1 / 1024 / 4096, and the literal 12N-variable QP at B = 4096.  Usage: tools/gpu_r3_breakdown.sh TAG
set -o pipefail
tag=${1:-r3bd}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for b in 1 1024 4096; do
  for v in default iter0 iter0s0 iter1 iter150 chk5; do
    timeout -k 10 120 python tools/perf_kernel.py $v $b 20 >> $out/breakdown.txt 2>&1 || { tail -5 $out/breakdown.txt; exit 1; }
  done
done
for v in default iter0 iter0s0 iter1 iter150 chk5; do
  LITERAL=1 timeout -k 10 120 python tools/perf_kernel.py $v 4096 10 >> $out/breakdown.txt 2>&1 || { tail -5 $out/breakdown.txt; exit 1; }
done
grep -v amdgpu.ids $out/breakdown.txt
