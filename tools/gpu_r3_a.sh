#!/bin/bash
# Round-3 opening run: GPU parity suite, smoke, headline bench line +
# kernel stats, force-QP line with fresh FETCH_SIZE / WRITE_SIZE passes
# (the round-1 traffic file predates the scratch fix).  Usage: tools/gpu_r3_a.sh TAG
set -o pipefail
tag=${1:-r3a}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -n 1 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/fetch -o run -- python tools/bench_qp.py --no-cpu-baseline --steps 3 --warmup 1 > $out/fetch.log 2>&1 || { tail -20 $out/fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $out/write -o run -- python tools/bench_qp.py --no-cpu-baseline --steps 3 --warmup 1 > $out/write.log 2>&1 || { tail -20 $out/write.log; exit 1; }
python tools/prof_summary.py traffic $out/fetch $out/write force_qp_kernel $out/traffic_force_qp_b65536.json && rm -rf $out/fetch $out/write
cp $out/traffic_force_qp_b65536.json profiles/traffic_force_qp_b65536.json
timeout -k 10 200 python tools/bench_qp.py > $out/bench_qp.json 2> $out/bench_qp.err || { tail -20 $out/bench_qp.err; exit 1; }
timeout -k 10 200 python tools/bench_qp.py --servo > $out/bench_servo.json 2> $out/bench_servo.err || { tail -20 $out/bench_servo.err; exit 1; }
cat $out/bench_qp.json $out/bench_servo.json
