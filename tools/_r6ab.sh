#!/bin/bash
# Force QP after the width setter: GI-core users' GPU tests (incl. the 8- vs
# 16-lane bit-identity test), default bench lines, servo block.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r6ab; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "force or hw_torque or servo or rt_ or body or gi or eiquadprog or qpsolver" > $out/pytest_force.log 2>&1 || { tail -30 $out/pytest_force.log; exit 1; }
tail -n 1 $out/pytest_force.log
for a in "--ticks 1" "--ticks 8" "--ticks 1 --ungrouped"; do
  timeout -k 10 200 python tools/bench_qp.py $a >> $out/bench_qp.jsonl 2>> $out/qp.err || { tail $out/qp.err; exit 1; }
done
python -c "
import json
for l in open('$out/bench_qp.jsonl'):
    d=json.loads(l); print(round(d['ms_per_step'],4), round(d['value']/1e6,1), d['config']['workload'][:120])"
timeout -k 10 200 python tools/bench_qp.py --servo > $out/servo.json 2>> $out/qp.err && cat $out/servo.json
