#!/bin/bash
# rt node tick: GPU parity tests + bench line + kernel stats.  Usage: tools/gpu_rt_quick.sh TAG
set -o pipefail
tag=${1:-rtq}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_rt_gpu.py tests/test_qp_gpu.py -x -v --timeout 150 --timeout-method thread > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
timeout -k 10 240 python tools/bench_rt.py --sets 10 --no-cpu-baseline > $out/bench_rt.json 2> $out/bench_rt.err || { tail -20 $out/bench_rt.err; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/kt -o run -- python tools/bench_rt.py --sets 10 --no-cpu-baseline --steps 30 > $out/kt.log 2>&1 || { tail -20 $out/kt.log; exit 1; }
tail -1 $out/pytest.log
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['ms_per_step']*1e3,1), 'us', '%.3g' % d['value'])" $out/bench_rt.json
python tools/prof_summary.py stats $out/kt $out/kt_stats.csv | head -5
