#!/bin/bash
# Round 3: one-wave kernel with N <= 10 LDS tables at 4 waves/SIMD vs the
# 3-wave build (variant w3 = -DQLOCO_SRBD_SHORT_WPE=0); GPU parity suite first.
set -o pipefail
tag=${1:-r3occ}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
BATCHES="4096 1024 8192 65536" tools/gpu_ab.sh $tag w3 || exit 1
