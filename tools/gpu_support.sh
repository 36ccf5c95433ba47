#!/bin/bash
# contact-phase flag: GPU parity tests, bench line, kernel trace
set -o pipefail
tag=${1:-sp}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_support_phase.py -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
timeout -k 10 240 python tools/bench_rt.py --support > $out/bench_support.json 2> $out/bench_support.err || { tail -20 $out/bench_support.err; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/kt -o run -- python tools/bench_rt.py --support --no-cpu-baseline --steps 20 > $out/kt.log 2>&1 || { tail -20 $out/kt.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/pf -o run -- python tools/bench_rt.py --support --no-cpu-baseline --steps 5 > $out/pf.log 2>&1 || { tail -20 $out/pf.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $out/pw -o run -- python tools/bench_rt.py --support --no-cpu-baseline --steps 5 > $out/pw.log 2>&1 || { tail -20 $out/pw.log; exit 1; }
tail -1 $out/pytest.log
cat $out/bench_support.json
python tools/prof_summary.py stats $out/kt $out/kt_stats.csv | head -3
python tools/prof_summary.py traffic $out/pf $out/pw support_phase $out/traffic.json && cat $out/traffic.json
