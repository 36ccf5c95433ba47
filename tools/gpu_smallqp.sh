#!/bin/bash
# small-QP + rt tick: GPU parity tests, bench lines, kernel traces.  Usage: tools/gpu_smallqp.sh TAG
set -o pipefail
tag=${1:-sq}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_qp_gpu.py tests/test_rt_gpu.py tests/test_host_gpu.py -x -v --timeout 150 --timeout-method thread > $out/pytest.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $out/pytest.log | tail -30; exit 1; }
timeout -k 10 300 python tools/bench_rt.py --no-cpu-baseline > $out/bench_rt.json 2> $out/bench_rt.err || { tail -20 $out/bench_rt.err; exit 1; }
timeout -k 10 300 python tools/bench_qp.py --no-cpu-baseline > $out/bench_qp.json 2> $out/bench_qp.err || { tail -20 $out/bench_qp.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt_rt -o run -- python tools/bench_rt.py --no-cpu-baseline --steps 30 > $out/kt_rt.log 2>&1 || { tail -20 $out/kt_rt.log; exit 1; }
grep -cE "PASSED" $out/pytest.log; cat $out/bench_rt.json $out/bench_qp.json
