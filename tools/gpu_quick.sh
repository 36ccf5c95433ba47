#!/bin/bash
# parity (SRBD + host shim) then the W=1 / W=2 timing points
set -o pipefail
out=${1:-gpurun_out/quick.log}
mkdir -p $(dirname $out)
timeout -k 10 400 python -m pytest tests/test_srbd_gpu.py tests/test_host_gpu.py -m gpu -x -q >> $out 2>&1 || exit 1
for b in 1024 4096 8192; do
  N=10 GAIT=trot timeout -k 10 120 python tools/perf_kernel.py default $b 5 >> $out 2>&1 || exit 1
done
N=10 GAIT=trot timeout -k 10 120 python tools/perf_kernel.py iter1 8192 5 >> $out 2>&1 || exit 1
N=16 GAIT=trot timeout -k 10 120 python tools/perf_kernel.py default 8192 5 >> $out 2>&1 || exit 1
grep -v amdgpu.ids $out
