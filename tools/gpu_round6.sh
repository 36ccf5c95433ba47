#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python -m pytest tests/test_srbd_gpu.py -x -q -m gpu > gpurun_out/r6/pytest.log 2>&1 || { tail -40 gpurun_out/r6/pytest.log; exit 1; }
for B in 256 4096 8192; do
  for v in iter1 iter150 default; do
    timeout -k 10 60 python tools/perf_kernel.py $v $B 10 >> gpurun_out/r6/scan.log 2>&1 || exit 1
  done
done
for v in iter1 default; do timeout -k 10 60 python tools/phase_timing.py $v 4096 >> gpurun_out/r6/phase.log 2>&1 || exit 1; done
tail -2 gpurun_out/r6/pytest.log; grep -v amdgpu.ids gpurun_out/r6/scan.log; grep -v amdgpu.ids gpurun_out/r6/phase.log
