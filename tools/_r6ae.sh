#!/bin/bash
# rt tick (body MPC on the GI core) and body-only bench: the session-start
# library (tools/_var/pregi, rev 975cc61) vs the current one, alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r6ae; mkdir -p $out
for k in 1 2; do
  for v in pregi cur; do
    if [ $v = pregi ]; then export QLOCO_LIB=$PWD/tools/_var/pregi/libqloco.so; else unset QLOCO_LIB; fi
    timeout -k 10 200 python tools/bench_rt.py --no-cpu-baseline > $out/rt.json 2>> $out/rt.err || { tail $out/rt.err; exit 1; }
    python -c "import json; d=json.load(open('$out/rt.json')); print('$v', round(d['ms_per_step']*1000,1), 'us', round(d['value']/1e6,1), 'M robot-ticks/s')" | tee -a $out/ab.txt
  done
done
# literal-mode parity tests with the 30 N one-check-apart u0 bound, and smoke
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "literal or lit" > $out/pytest_literal.log 2>&1 || { tail -30 $out/pytest_literal.log; exit 1; }
tail -n 1 $out/pytest_literal.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
# literal headline breakdown (tools/perf_kernel.py, B = 4096, 100 launches each after 2)
for v in default iter0 iter0s0 iter1 iter150 default; do
  LITERAL=1 timeout -k 10 120 python tools/perf_kernel.py $v 4096 100 >> $out/breakdown.txt 2>> $out/pk.err || { tail $out/pk.err; exit 1; }
done
cat $out/breakdown.txt
