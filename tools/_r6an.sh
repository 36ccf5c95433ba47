#!/bin/bash
# body MPC with s(x) also in LDS (serial scans read LDS) vs HEAD (tools/_var/preslds)
# serial): GI-user GPU tests, force QP and rt tick against tools/_var/preslds
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r6an; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "force or hw_torque or servo or rt_ or body or gi or eiquadprog or qpsolver" > $out/pytest_gi.log 2>&1 || { tail -30 $out/pytest_gi.log; exit 1; }
tail -n 1 $out/pytest_gi.log
for k in 1 2; do
  for v in pre cur; do
    if [ $v = pre ]; then export QLOCO_LIB=$PWD/tools/_var/preslds/libqloco.so; else unset QLOCO_LIB; fi
    timeout -k 10 200 python tools/bench_qp.py --no-cpu-baseline > $out/q.json 2>> $out/err.txt || { tail $out/err.txt; exit 1; }
    timeout -k 10 200 python tools/bench_qp.py --no-cpu-baseline --ticks 8 > $out/q8.json 2>> $out/err.txt || { tail $out/err.txt; exit 1; }
    timeout -k 10 200 python tools/bench_rt.py --no-cpu-baseline > $out/rt.json 2>> $out/err.txt || { tail $out/err.txt; exit 1; }
    python -c "
import json
q=json.load(open('$out/q.json')); q8=json.load(open('$out/q8.json')); r=json.load(open('$out/rt.json'))
print('$v', 'force %.4f ms' % q['ms_per_step'], 'force(8 ticks) %.4f ms' % q8['ms_per_step'], 'rt %.1f us' % (r['ms_per_step']*1000))" | tee -a $out/ab.txt
  done
done
unset QLOCO_LIB
timeout -k 10 200 python tools/bench_qp.py > $out/bench_qp.json 2>> $out/err.txt && cat $out/bench_qp.json | cut -c1-200
timeout -k 10 200 python tools/bench_qp.py --servo --no-cpu-baseline > $out/servo.json 2>> $out/err.txt && cat $out/servo.json | cut -c1-200
