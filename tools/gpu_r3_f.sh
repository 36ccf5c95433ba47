#!/bin/bash
# Round-3 run F: full GPU suite, headline bench (with the literal line),
# parity scans of the shipped Gauss-Jordan form (reduced + literal).
set -o pipefail
tag=${1:-r3f}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
grep -E "^E  .*assert|FAILED" $out/pytest_gpu.log | head -30; tail -1 $out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 400 python -u tools/srbd_parity_scan.py > $out/scan_reduced.txt 2>&1 || { tail -20 $out/scan_reduced.txt; exit 1; }
timeout -k 10 400 python -u tools/srbd_parity_scan.py --literal 10 64 trot 1e-3 10 48 mixed 1e-3 16 24 trot 1e-3 10 24 trot 1e-6 16 16 mixed 1e-5 > $out/scan_literal.txt 2>&1 || { tail -20 $out/scan_literal.txt; exit 1; }
grep -E "==|wrench" $out/scan_reduced.txt $out/scan_literal.txt
exit 0
