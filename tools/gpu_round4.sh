#!/bin/bash
# counters + batch scan for the SRBD kernel
set -o pipefail
mkdir -p gpurun_out/r4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for B in 256 1024 2048 4096 8192; do
  for v in iter1 default; do
    timeout -k 10 60 python tools/perf_kernel.py $v $B 10 >> gpurun_out/r4/scan.log 2>&1 || exit 1
  done
done
timeout -k 10 60 rocprofv3 -L > gpurun_out/r4/counters.txt 2>&1 || true
for v in iter1 default; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/r4/pmc1_$v -o run -- python tools/perf_kernel.py $v 4096 3 > gpurun_out/r4/pmc1_$v.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d gpurun_out/r4/pmc2_$v -o run -- python tools/perf_kernel.py $v 4096 3 > gpurun_out/r4/pmc2_$v.log 2>&1 || exit 1
done
cat gpurun_out/r4/scan.log
