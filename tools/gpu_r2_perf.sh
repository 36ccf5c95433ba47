#!/bin/bash
# SRBD perf points: bench line, batch scan and configs 3-5 per-GPU shares.  Usage: tools/gpu_r2_perf.sh TAG
set -o pipefail
tag=${1:-r2p}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
for b in 1024 4096 8192; do
  N=10 GAIT=trot timeout -k 10 120 python tools/perf_kernel.py default $b 10 >> $out/scan.txt 2>&1 || exit 1
done
N=16 GAIT=trot timeout -k 10 120 python tools/perf_kernel.py default 65536 3 >> $out/scan.txt 2>&1 || exit 1
N=20 GAIT=pace timeout -k 10 120 python tools/perf_kernel.py default 65536 3 >> $out/scan.txt 2>&1 || exit 1
N=10 GAIT=mixed timeout -k 10 120 python tools/perf_kernel.py default 131072 3 >> $out/scan.txt 2>&1 || exit 1
grep -v amdgpu.ids $out/scan.txt
