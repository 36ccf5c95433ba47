#!/bin/bash
# MFMA block-GJ inverse in srbd_admm_kernel<1>: GPU parity suite, A/B against
# the DPP Gauss-Jordan build (tools/_var/dppinv), bench line, kernel stats.
# Usage: tools/gpu_r2_mfma.sh TAG
set -o pipefail
tag=${1:-r2m}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
for b in 1 1024 4096 8192 65536; do
  for v in default iter0 iter150; do
    timeout -k 10 120 python tools/perf_kernel.py $v $b 5 >> $out/scan.txt 2>&1 || { tail -5 $out/scan.txt; exit 1; }
    QLOCO_LIB=tools/_var/dppinv/libqloco.so timeout -k 10 120 python tools/perf_kernel.py $v $b 5 >> $out/scan.txt 2>&1 || { tail -5 $out/scan.txt; exit 1; }
  done
done
grep -v amdgpu.ids $out/scan.txt
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/ktrace -o run -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $out/ktrace.log 2>&1 || { tail -20 $out/ktrace.log; exit 1; }
find $out/ktrace -name "*kernel_stats.csv" -exec cat {} \; | head -5
