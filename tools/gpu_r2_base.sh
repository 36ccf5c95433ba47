#!/bin/bash
# Round-2 opening measurement: GPU parity suite, bench line, rocprofv3 stats,
# SQ counter passes on the shipped SRBD kernel.  Usage: tools/gpu_r2_base.sh TAG
set -o pipefail
tag=${1:-r2a}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/ktrace -o run -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $out/ktrace.log 2>&1 || { tail -20 $out/ktrace.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $out/pmc1 -o run -- python tools/perf_kernel.py default 4096 3 > $out/pmc1.log 2>&1 || { tail -20 $out/pmc1.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $out/pmc2 -o run -- python tools/perf_kernel.py default 4096 3 > $out/pmc2.log 2>&1 || { tail -20 $out/pmc2.log; exit 1; }
for b in 1024 2048 4096 8192; do
  N=10 GAIT=trot timeout -k 10 120 python tools/perf_kernel.py default $b 10 >> $out/scan.txt 2>&1 || exit 1
  N=10 GAIT=trot timeout -k 10 120 python tools/perf_kernel.py iter150 $b 10 >> $out/scan.txt 2>&1 || exit 1
done
cat $out/scan.txt
