#!/bin/bash
# Persistent atomic-queue grid (QLOCO_SRBD_PQ=1) and occupancy variants of
# srbd_admm_kernel<1> against the product launch.  Usage: tools/gpu_r2_pq.sh TAG
set -o pipefail
tag=${1:-r2q}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_srbd_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_srbd.log 2>&1 || { tail -40 $out/pytest_srbd.log; exit 1; }
QLOCO_SRBD_PQ=1 timeout -k 10 300 python -u -m pytest tests/test_srbd_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_srbd_pq.log 2>&1 || { tail -40 $out/pytest_srbd_pq.log; exit 1; }
tail -n 1 $out/pytest_srbd.log $out/pytest_srbd_pq.log
for b in 1024 2048 4096 8192 16384 65536; do
  timeout -k 10 120 python tools/perf_kernel.py default $b 10 >> $out/scan.txt 2>&1 || exit 1
  QLOCO_SRBD_PQ=1 timeout -k 10 120 python tools/perf_kernel.py default $b 10 | sed 's/^prod /PQ   /' >> $out/scan.txt 2>&1 || exit 1
  for v in wpe3 wpe4; do
    QLOCO_LIB=tools/_var/$v/libqloco.so timeout -k 10 120 python tools/perf_kernel.py default $b 10 >> $out/scan.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $out/scan.txt
