#!/bin/bash
set -o pipefail
tag=${1:-r2h}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_qp_gpu.py tests/test_servo_gpu.py tests/test_rt_gpu.py tests/test_host_gpu.py "tests/test_srbd_gpu.py::test_srbd_config5_share_sampled_against_oracle" -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gi.log 2>&1 || { tail -40 $out/pytest_gi.log; exit 1; }
tail -n 1 $out/pytest_gi.log
timeout -k 10 200 python tools/bench_qp.py --no-cpu-baseline > $out/bench_qp.json 2> $out/bench_qp.err || { tail -20 $out/bench_qp.err; exit 1; }
timeout -k 10 200 python tools/bench_qp.py --servo --no-cpu-baseline > $out/bench_servo.json 2> $out/bench_servo.err || { tail -20 $out/bench_servo.err; exit 1; }
timeout -k 10 200 python tools/bench_rt.py --no-cpu-baseline > $out/bench_rt.json 2> $out/bench_rt.err || { tail -20 $out/bench_rt.err; exit 1; }
for f in bench_qp bench_servo bench_rt; do python -c "import json; d=json.load(open('$out/$f.json')); print('$f', d['value'], d['ms_per_step'])"; done
