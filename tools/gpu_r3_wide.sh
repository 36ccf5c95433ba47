#!/bin/bash
# Wide-kernel half-width buckets (HC = 96/112/120): GPU parity suite, then
# same-call A/B against the previous tree (tools/_var/r3head) on the wide
# workloads (literal N = 16 / 20, stand-balance N = 16 / 20).
set -o pipefail
tag=${1:-r3wide}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { grep -E "^FAILED|Error|assert" $out/pytest_gpu.log | tail -30; exit 1; }
tail -n 1 $out/pytest_gpu.log
for rep in 1 2; do
  GAIT=trot N=16 timeout -k 10 180 python tools/perf_kernel.py default 65536 3 >> $out/ab.txt 2>&1 || exit 1
  GAIT=trot N=16 QLOCO_LIB=tools/_var/c9w2/libqloco.so timeout -k 10 180 python tools/perf_kernel.py default 65536 3 >> $out/ab.txt 2>&1 || exit 1
  for w in "trot 16 8192 1" "pace 20 8192 1" "stance 16 8192 0" "stance 20 8192 0"; do
    set -- $w
    for L in "" tools/_var/r3head/libqloco.so; do
      GAIT=$1 N=$2 LITERAL=$4 QLOCO_LIB=$L timeout -k 10 180 python tools/perf_kernel.py default $3 3 >> $out/ab.txt 2>&1 || { tail -5 $out/ab.txt; exit 1; }
    done
  done
done
grep -v amdgpu.ids $out/ab.txt
