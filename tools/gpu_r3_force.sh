#!/bin/bash
# Force-QP occupancy: GI / force / servo parity tests, then same-call A/B of
# the product library against variants (tools/variant_lib.py) on
# tools/bench_qp.py.  Usage: tools/gpu_r3_force.sh TAG VARIANT...
set -o pipefail
tag=${1:-r3force}; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_qp_gpu.py tests/test_servo_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_qp.log 2>&1 || { tail -40 $out/pytest_qp.log; exit 1; }
tail -n 1 $out/pytest_qp.log
for rep in 1 2; do
  timeout -k 10 200 python tools/bench_qp.py --no-cpu-baseline > $out/qp_prod_$rep.json 2>> $out/qp.err || { tail -20 $out/qp.err; exit 1; }
  python -c "import json; d=json.load(open('$out/qp_prod_$rep.json')); print('prod', d['ms_per_step'], round(d['value']/1e6,2), 'M/s')"
  for v in "$@"; do
    QLOCO_LIB=tools/_var/$v/libqloco.so timeout -k 10 200 python tools/bench_qp.py --no-cpu-baseline > $out/qp_${v}_$rep.json 2>> $out/qp.err || { tail -20 $out/qp.err; exit 1; }
    python -c "import json; d=json.load(open('$out/qp_${v}_$rep.json')); print('$v', d['ms_per_step'], round(d['value']/1e6,2), 'M/s')"
  done
done
