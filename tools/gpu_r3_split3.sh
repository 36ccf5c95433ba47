#!/bin/bash
# Split kernel iteration: GPU parity suite, then same-call A/B vs row4 / w3.
set -o pipefail
tag=${1:-r3split3}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
BATCHES="${BATCHES:-4096 1024 65536}" tools/gpu_ab.sh $tag ${VARIANTS:-row4} || exit 1
