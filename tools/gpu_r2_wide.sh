#!/bin/bash
# Wide SRBD kernel (43..80 stance legs): new GPU tests, the SRBD GPU file, perf points.
# Usage: tools/gpu_r2_wide.sh TAG
set -o pipefail
tag=${1:-r2w}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_srbd_gpu.py -x -v --timeout 200 --timeout-method thread -k "wide or three_kernel" > $out/pytest_wide.log 2>&1 || { tail -60 $out/pytest_wide.log; exit 1; }
tail -8 $out/pytest_wide.log
for cfg in "12 stance 4096" "16 stance 8192" "20 stance 8192" "20 mixed 8192"; do
  set -- $cfg
  N=$1 GAIT=$2 timeout -k 10 120 python tools/perf_kernel.py default $3 3 >> $out/scan.txt 2>&1 || { tail -20 $out/scan.txt; exit 1; }
done
grep -v amdgpu.ids $out/scan.txt
timeout -k 10 600 python -u -m pytest tests/test_srbd_gpu.py -x -q --timeout 300 --timeout-method thread > $out/pytest_srbd.log 2>&1 || { tail -40 $out/pytest_srbd.log; exit 1; }
tail -3 $out/pytest_srbd.log
