#!/bin/bash
# Spill-free force_qp_kernel (two waves/SIMD): GI / force / servo parity
# tests, bench lines (force QP, servo block) and fresh HBM traffic.
# Usage: tools/gpu_r3_force2.sh TAG
set -o pipefail
tag=${1:-r3f2}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_qp_gpu.py tests/test_servo_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_qp.log 2>&1 || { tail -40 $out/pytest_qp.log; exit 1; }
tail -n 1 $out/pytest_qp.log
for rep in 1 2; do
  timeout -k 10 200 python tools/bench_qp.py > $out/bench_qp_$rep.json 2>> $out/qp.err || { tail -20 $out/qp.err; exit 1; }
  python -c "import json; d=json.load(open('$out/bench_qp_$rep.json')); print('force', d['ms_per_step'], round(d['value']/1e6,2), 'M/s')"
done
timeout -k 10 200 python tools/bench_qp.py --servo --no-cpu-baseline > $out/bench_servo.json 2>> $out/qp.err || { tail -20 $out/qp.err; exit 1; }
python -c "import json; d=json.load(open('$out/bench_servo.json')); print('servo', d['ms_per_step'], round(d['value']/1e6,2), 'M/s')"
bash tools/gpu_r3_force_traffic.sh $tag
