#!/bin/bash
# small-QP paths: force QP bench line + kernel trace.  Usage: tools/gpu_qp.sh TAG
set -o pipefail
tag=${1:-qp}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/bench_qp.py > $out/bench_qp.json 2> $out/bench_qp.err || { tail -20 $out/bench_qp.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt_qp -o run -- python tools/bench_qp.py --no-cpu-baseline --steps 30 > $out/kt_qp.log 2>&1 || { tail -20 $out/kt_qp.log; exit 1; }
cat $out/bench_qp.json
