#!/bin/bash
# HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes) of the two-wave
# C2 = 3 / C2 = 6 buckets on the mixed config-5 share (131,072 instances),
# shipped library (both buckets at four waves/SIMD for N <= 10) and the
# C2 = 6 three-wave variant (tools/_var/c6w3).  Usage: tools/gpu_r3_w2_traffic.sh TAG
set -o pipefail
tag=${1:-r3wt}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in cur c6w3; do
  L=""; [ $lib = c6w3 ] && L=tools/_var/c6w3/libqloco.so
  for ctr in FETCH_SIZE WRITE_SIZE; do
    QLOCO_LIB=$L GAIT=mixed N=10 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d $out/${lib}_$ctr -o run -- python tools/perf_kernel.py default 131072 2 > $out/${lib}_$ctr.log 2>&1 || { tail -20 $out/${lib}_$ctr.log; exit 1; }
  done
  for k in "2, 4, false, 10, 3>" "2, 4, false, 10, 6>" "2, 3, false, 20, 6>"; do
    echo "$lib kernel <$k" >> $out/traffic.txt
    python tools/prof_summary.py traffic $out/${lib}_FETCH_SIZE $out/${lib}_WRITE_SIZE "$k" $out/tmp.json 2>&1 | tr -d '\n' >> $out/traffic.txt
    echo >> $out/traffic.txt
  done
  rm -rf $out/${lib}_FETCH_SIZE $out/${lib}_WRITE_SIZE
done
cat $out/traffic.txt
