#!/bin/bash
# Measurement of the 8f rows beside the headline: rt node tick and force QP
# bench lines (with CPU baselines), rocprofv3 kernel stats, HBM traffic PMC
# passes (FETCH_SIZE / WRITE_SIZE in separate runs).  Usage: tools/gpu_rows.sh TAG
set -o pipefail
tag=${1:-rows}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/bench_rt.py > $out/bench_rt.json 2> $out/bench_rt.err || { tail -20 $out/bench_rt.err; exit 1; }
timeout -k 10 300 python tools/bench_qp.py > $out/bench_qp.json 2> $out/bench_qp.err || { tail -20 $out/bench_qp.err; exit 1; }
for b in rt qp; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/kt_$b -o run -- python tools/bench_$b.py --no-cpu-baseline --steps 30 > $out/kt_$b.log 2>&1 || { tail -20 $out/kt_$b.log; exit 1; }
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/pf_$b -o run -- python tools/bench_$b.py --no-cpu-baseline --steps 10 > $out/pf_$b.log 2>&1 || { tail -20 $out/pf_$b.log; exit 1; }
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $out/pw_$b -o run -- python tools/bench_$b.py --no-cpu-baseline --steps 10 > $out/pw_$b.log 2>&1 || { tail -20 $out/pw_$b.log; exit 1; }
done
cat $out/bench_rt.json $out/bench_qp.json
