#!/bin/bash
# Full GPU parity suite + bench line + SRBD batch scan.  Usage: tools/gpu_r2_check.sh TAG
set -o pipefail
tag=${1:-r2x}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
for b in 1024 4096 8192; do
  N=10 GAIT=trot timeout -k 10 120 python tools/perf_kernel.py default $b 10 >> $out/scan.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $out/scan.txt
