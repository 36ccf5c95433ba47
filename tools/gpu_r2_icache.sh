#!/bin/bash
# Setup-cost ablations (production build) and instruction-cache counters of
# the SRBD kernel.  Usage: tools/gpu_r2_icache.sh TAG
set -o pipefail
tag=${1:-r2i}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 -L > $out/counters.txt 2>&1 || true
grep -i -E "ICACHE|IFETCH|INST_CACHE|SQC_" $out/counters.txt | head -60 > $out/counters_icache.txt || true
for b in 1 1024 4096; do
  for v in default iter0 iter0s0 iter1 iter150 iter150s0; do
    timeout -k 10 120 python tools/perf_kernel.py $v $b 10 >> $out/scan.txt 2>&1 || { tail -20 $out/scan.txt; exit 1; }
  done
done
cat $out/scan.txt
cat $out/counters_icache.txt
