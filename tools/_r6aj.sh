#!/bin/bash
# force-QP graph replay test + the force / servo group
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r6aj; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_qp_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_qp.log 2>&1 || { tail -40 $out/pytest_qp.log; exit 1; }
tail -n 3 $out/pytest_qp.log
