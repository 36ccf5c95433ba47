#!/bin/bash
# rt tick steady state: kernel stats over the 100 timed ticks only (after 150 warm-up ticks)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/r6ak; mkdir -p $out
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/kt -o run -- python tools/bench_rt.py --no-cpu-baseline > $out/kt.log 2>&1 || { tail $out/kt.log; exit 1; }
python tools/db_kernel_stats.py $out/kt --last 100 > $out/kernel_stats_rt_steady.csv && rm -rf $out/kt
cat $out/kernel_stats_rt_steady.csv
tail -1 $out/kt.log | cut -c1-300
