#!/bin/bash
# Full GPU validation + measurement: pytest -m gpu, smoke, bench JSON,
# rocprofv3 kernel-trace stats (csv), HBM traffic PMC passes.  Usage: tools/gpu_full.sh TAG
set -o pipefail
tag=${1:-r1}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/ktrace -o run -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $out/ktrace.log 2>&1 || { tail -20 $out/ktrace.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/pmc_fetch -o run -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $out/pmc_fetch.log 2>&1 || { tail -20 $out/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $out/pmc_write -o run -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $out/pmc_write.log 2>&1 || { tail -20 $out/pmc_write.log; exit 1; }
tail -2 $out/pytest_gpu.log; tail -1 $out/smoke.log; cat $out/bench.json
find $out/ktrace -name "*.csv"
# §8f row 4: leg kinematics bench + kernel trace
timeout -k 10 300 python tools/bench_kin.py > $out/bench_kin.json 2> $out/bench_kin.err || { tail -20 $out/bench_kin.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/ktrace_kin -o run -- python tools/bench_kin.py --no-cpu-baseline > $out/ktrace_kin.log 2>&1 || { tail -20 $out/ktrace_kin.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/pmc_kin_fetch -o run -- python tools/bench_kin.py --no-cpu-baseline --steps 10 > $out/pmc_kin_fetch.log 2>&1 || { tail -20 $out/pmc_kin_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $out/pmc_kin_write -o run -- python tools/bench_kin.py --no-cpu-baseline --steps 10 > $out/pmc_kin_write.log 2>&1 || { tail -20 $out/pmc_kin_write.log; exit 1; }
cat $out/bench_kin.json
