#!/bin/bash
# Force QP group width A/B with s(x), u/A snapshots and the iai/iaexcl flags in registers (19.8 KB per 8-robot block, 8 per CU): forced
# 8 / 16 and the shipped default (8); GI-core users'
# tests first (force, servo, body, generic EiQuadProg).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r6ac; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "force or hw_torque or servo or rt_ or body or gi or eiquadprog or qpsolver" > $out/pytest_force.log 2>&1 || { tail -30 $out/pytest_force.log; exit 1; }
tail -n 1 $out/pytest_force.log
for gw in 8 16 default 8 16 default; do
  for a in "--ticks 1" "--ticks 8" "--ticks 1 --ungrouped"; do
    if [ $gw = default ]; then unset QLOCO_FORCE_GW; else export QLOCO_FORCE_GW=$gw; fi
    timeout -k 10 200 python tools/bench_qp.py --no-cpu-baseline $a > $out/q.json 2>> $out/qp.err || { tail $out/qp.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$out/q.json')); print('gw=$gw', round(d['ms_per_step'],4), d['config']['workload'])" | tee -a $out/ab.txt
  done
done
unset QLOCO_FORCE_GW
timeout -k 10 200 python tools/bench_qp.py --servo --no-cpu-baseline > $out/servo.json 2>> $out/qp.err && cat $out/servo.json
bash tools/gpu.sh r6ac sqqp || exit 1
