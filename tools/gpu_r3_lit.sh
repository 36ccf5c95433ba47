#!/bin/bash
# Literal full-QP mode: parity envelope scan vs the full-QP restatement, then
# the literal GPU tests.  Usage: tools/gpu_r3_lit.sh TAG
set -o pipefail
tag=${1:-r3lit}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u tools/srbd_parity_scan.py --literal 10 64 trot 1e-3 10 48 pace 1e-3 10 48 mixed 1e-3 16 16 trot 1e-3 20 12 pace 1e-3 4 32 trot 1e-3 10 24 trot 1e-6 > $out/scan_literal.txt 2>&1 || { tail -30 $out/scan_literal.txt; exit 1; }
cat $out/scan_literal.txt
timeout -k 10 600 python -u -m pytest tests/test_srbd_gpu.py -v --timeout 300 --timeout-method thread -k "literal" > $out/pytest_lit.log 2>&1; tail -15 $out/pytest_lit.log
