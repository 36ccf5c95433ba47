#!/bin/bash
# Round 3: column-split one-wave kernel (product) vs the row layout at four
# waves/SIMD (row4) and at three (w3); GPU parity suite first, SIMD trace.
set -o pipefail
tag=${1:-r3split}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
BATCHES="4096 1024 65536" tools/gpu_ab.sh $tag row4 w3 || exit 1
QLOCO_LIB=tools/_var/trace5/libqloco.so timeout -k 10 120 python tools/simd_trace.py 4096 $out/trace_4096.npz > $out/trace_4096.txt 2>&1 || exit 1
grep -v amdgpu.ids $out/trace_4096.txt | head -8
