#!/bin/bash
# HBM traffic of the shipped force_qp_kernel<8> (grouped launch, 65,536
# robots; FETCH_SIZE and WRITE_SIZE in separate --pmc passes) and a kernel
# trace of the force-QP bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/r6ah; mkdir -p $out
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/fetch -o run -- python tools/bench_qp.py --steps 3 --warmup 2 --no-cpu-baseline > $out/fetch.log 2>&1 || { tail $out/fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $out/write -o run -- python tools/bench_qp.py --steps 3 --warmup 2 --no-cpu-baseline > $out/write.log 2>&1 || { tail $out/write.log; exit 1; }
python tools/prof_summary.py traffic $out/fetch $out/write force_qp_kernel $out/traffic_force_qp_b65536.json && rm -rf $out/fetch $out/write
cat $out/traffic_force_qp_b65536.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/kt -o run -- python tools/bench_qp.py --no-cpu-baseline > $out/kt.log 2>&1 || { tail $out/kt.log; exit 1; }
python tools/db_kernel_stats.py $out/kt > $out/kernel_stats_force_qp.csv && rm -rf $out/kt
cat $out/kernel_stats_force_qp.csv
