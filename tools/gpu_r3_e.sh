#!/bin/bash
# Round-3 run E: literal NaN diagnostic + full GPU suite + headline bench + A/B.
set -o pipefail
tag=${1:-r3e}; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/literal_nan_diag.py > $out/nan_diag.txt 2>&1 || { tail -20 $out/nan_diag.txt; exit 1; }
grep literal $out/nan_diag.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1; grep -E "^E  .*assert|FAILED" $out/pytest_gpu.log | head -30; tail -1 $out/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
[ $# -gt 0 ] && bash tools/gpu_ab.sh $tag "$@"
exit 0
