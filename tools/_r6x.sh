#!/bin/bash
# Force QP group width A/B: 8-lane groups (default) vs 16-lane (QLOCO_FORCE_GW=16),
# bit-identity tests first.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r6x; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "force or hw_torque or servo or rt_ or body" > $out/pytest_force.log 2>&1 || { tail -30 $out/pytest_force.log; exit 1; }
tail -n 1 $out/pytest_force.log
for gw in 8 16 8 16; do
  for a in "--ticks 1" "--ticks 8" "--ticks 1 --ungrouped"; do
    QLOCO_FORCE_GW=$gw timeout -k 10 200 python tools/bench_qp.py --no-cpu-baseline $a > $out/q.json 2>> $out/qp.err || { tail $out/qp.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$out/q.json')); print('gw=$gw', round(d['ms_per_step'],4), d['config']['workload'])" | tee -a $out/ab.txt
  done
done
