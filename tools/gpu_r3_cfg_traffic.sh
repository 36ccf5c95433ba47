#!/bin/bash
# HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes) of the two-wave
# C2 = 9 / C2 = 15 buckets on configs 3 and 4 (N = 16 trot, N = 20 pace,
# 65,536 instances).  Usage: tools/gpu_r3_cfg_traffic.sh TAG
set -o pipefail
tag=${1:-r3ct}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for w in "trot 16 9>" "pace 20 15>"; do
  set -- $w
  for ctr in FETCH_SIZE WRITE_SIZE; do
    GAIT=$1 N=$2 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d $out/$1_$ctr -o run -- python tools/perf_kernel.py default 65536 2 > $out/$1_$ctr.log 2>&1 || { tail -20 $out/$1_$ctr.log; exit 1; }
  done
  echo "$1 N=$2 kernel srbd_admm_kernel<2, 3, false, 20, $3" >> $out/traffic.txt
  python tools/prof_summary.py traffic $out/$1_FETCH_SIZE $out/$1_WRITE_SIZE "false, 20, $3" $out/tmp.json 2>&1 | tr -d '\n' >> $out/traffic.txt
  echo >> $out/traffic.txt
  rm -rf $out/$1_FETCH_SIZE $out/$1_WRITE_SIZE
done
cat $out/traffic.txt
