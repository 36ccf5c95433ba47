#!/bin/bash
# Round-3 run D: SRBD parity suite after the code-size restructuring, then
# the same-call A/B of the product library vs variants.
set -o pipefail
tag=${1:-r3d}; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests/test_srbd_gpu.py tests/test_host_gpu.py -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1; grep -E "^E  .*assert|FAILED" $out/pytest.log | head -30; tail -1 $out/pytest.log
bash tools/gpu_ab.sh $tag "$@"
