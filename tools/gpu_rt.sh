#!/bin/bash
# rt node tick: GPU parity tests, bench line, kernel trace.
# Usage: tools/gpu_rt.sh TAG
set -o pipefail
tag=${1:-rt}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_rt_gpu.py -x -v -s --timeout 150 --timeout-method thread > $out/pytest_rt.log 2>&1 || { tail -40 $out/pytest_rt.log; exit 1; }
timeout -k 10 300 python tools/bench_rt.py > $out/bench_rt.json 2> $out/bench_rt.err || { tail -20 $out/bench_rt.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt_rt -o run -- python tools/bench_rt.py --no-cpu-baseline --steps 30 > $out/kt_rt.log 2>&1 || { tail -20 $out/kt_rt.log; exit 1; }
grep -E "passed|failed|parity" $out/pytest_rt.log; cat $out/bench_rt.json
