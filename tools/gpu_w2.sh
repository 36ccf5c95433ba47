#!/bin/bash
# W=2 (N=16 trot) timing sweep + the W=1 headline point, for before/after.
set -o pipefail
out=${1:-gpurun_out/w2.log}
mkdir -p $(dirname $out)
timeout -k 10 300 python -m pytest tests/test_srbd_gpu.py -m gpu -x -q >> $out 2>&1 || exit 1
for v in iter1 default; do
  N=16 GAIT=trot timeout -k 10 120 python tools/perf_kernel.py $v 8192 5 >> $out 2>&1 || exit 1
  N=16 GAIT=trot timeout -k 10 120 python tools/perf_kernel.py $v 256 5 >> $out 2>&1 || exit 1
done
N=10 GAIT=trot timeout -k 10 120 python tools/perf_kernel.py default 4096 5 >> $out 2>&1 || exit 1
grep -v amdgpu.ids $out
