#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r6q; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt -o run -- python bench.py --steps 30 --warmup 5 --no-second-line --no-cpu-baseline --prewarm 20 > $out/kt.log 2>&1 || { tail $out/kt.log; exit 1; }
python tools/db_kernel_stats.py $out/kt --last 30 > $out/kernel_stats_capped.csv && rm -rf $out/kt
head -4 $out/kernel_stats_capped.csv
