#!/bin/bash
# body MPC on 8-lane groups: body / rt GPU tests, then the rt tick against
# the session-start library (tools/_var/pregi, rev 975cc61), alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r6af; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "body or rt_ or replay or node or indexfind or support" > $out/pytest_body.log 2>&1 || { tail -30 $out/pytest_body.log; exit 1; }
tail -n 1 $out/pytest_body.log
for k in 1 2; do
  for v in pregi cur; do
    if [ $v = pregi ]; then export QLOCO_LIB=$PWD/tools/_var/pregi/libqloco.so; else unset QLOCO_LIB; fi
    timeout -k 10 200 python tools/bench_rt.py --no-cpu-baseline > $out/rt.json 2>> $out/rt.err || { tail $out/rt.err; exit 1; }
    python -c "import json; d=json.load(open('$out/rt.json')); print('$v', round(d['ms_per_step']*1000,1), 'us', round(d['value']/1e6,1), 'M robot-ticks/s')" | tee -a $out/ab.txt
  done
done
unset QLOCO_LIB
timeout -k 10 200 python tools/bench_rt.py > $out/bench_rt.json 2>> $out/rt.err && cat $out/bench_rt.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/kt -o run -- python tools/bench_rt.py --no-cpu-baseline --steps 50 --warmup 50 > $out/kt.log 2>&1 || { tail $out/kt.log; exit 1; }
python tools/db_kernel_stats.py $out/kt > $out/kernel_stats_rt.csv && rm -rf $out/kt
cat $out/kernel_stats_rt.csv
