#!/bin/bash
# GPU parity suite + per-phase cycle counts of the SRBD kernel (phase-timing
# build, tools/phase_timing.py).  Usage: tools/gpu_r2_phase.sh TAG
set -o pipefail
tag=${1:-r2p}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
for v in "default 1" "default 1024" "iter150 1024" "default 4096" "iter150 4096"; do
  timeout -k 10 120 python tools/phase_timing.py $v >> $out/phase.txt 2>&1 || { tail -20 $out/phase.txt; exit 1; }
done
cat $out/phase.txt
