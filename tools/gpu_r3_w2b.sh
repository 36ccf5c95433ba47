#!/bin/bash
# Two-wave column buckets (C2 = 3/6/9/16 kernel instantiations): GPU parity
# suite, then same-call A/B against the previous tree (tools/_var/r3head) on
# the two-wave workloads.  Usage: tools/gpu_r3_w2b.sh TAG
set -o pipefail
tag=${1:-r3w2b}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -n 1 $out/pytest_gpu.log
for rep in 1 2; do
  for w in "mixed 10 131072 0" "trot 16 65536 0" "pace 20 65536 0" "trot 10 4096 1" "trot 10 4096 0"; do
    set -- $w
    for L in "" tools/_var/r3head/libqloco.so; do
      GAIT=$1 N=$2 LITERAL=$4 QLOCO_LIB=$L timeout -k 10 180 python tools/perf_kernel.py default $3 5 >> $out/ab.txt 2>&1 || { tail -5 $out/ab.txt; exit 1; }
    done
  done
done
grep -v amdgpu.ids $out/ab.txt
