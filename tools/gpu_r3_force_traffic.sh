#!/bin/bash
# Fresh HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the
# shipped force_qp_kernel at 65,536 robots.  Usage: tools/gpu_r3_force_traffic.sh TAG
set -o pipefail
tag=${1:-r3ft}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/fetch -o run -- python tools/bench_qp.py --steps 3 --warmup 1 --no-cpu-baseline > $out/fetch.log 2>&1 || { tail -20 $out/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $out/write -o run -- python tools/bench_qp.py --steps 3 --warmup 1 --no-cpu-baseline > $out/write.log 2>&1 || { tail -20 $out/write.log; exit 1; }
python tools/prof_summary.py traffic $out/fetch $out/write force_qp $out/traffic_force_qp_b65536.json > /dev/null
rm -rf $out/fetch $out/write
cat $out/traffic_force_qp_b65536.json
