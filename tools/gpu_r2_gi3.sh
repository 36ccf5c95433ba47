#!/bin/bash
set -o pipefail
tag=${1:-r2h}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_qp_gpu.py tests/test_servo_gpu.py tests/test_rt_gpu.py tests/test_host_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gi.log 2>&1 || { tail -40 $out/pytest_gi.log; exit 1; }
tail -n 1 $out/pytest_gi.log
QLOCO_LIB=tools/_var/giphase/libqloco.so timeout -k 10 120 python tools/gi_phase.py 65536 > $out/gi_phase.txt 2>&1 || { tail -20 $out/gi_phase.txt; exit 1; }
grep -v amdgpu.ids $out/gi_phase.txt
timeout -k 10 200 python tools/bench_qp.py --no-cpu-baseline > $out/bench_qp.json 2> $out/bench_qp.err || { tail -20 $out/bench_qp.err; exit 1; }
cat $out/bench_qp.json
timeout -k 10 200 python tools/bench_rt.py --no-cpu-baseline > $out/bench_rt.json 2> $out/bench_rt.err || { tail -20 $out/bench_rt.err; exit 1; }
cat $out/bench_rt.json
