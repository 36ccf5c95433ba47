#!/bin/bash
# Same-call A/B of the product library against variant libraries
# (tools/variant_lib.py NAME ...) on the headline workload and neighbours.
# Usage: tools/gpu_ab.sh TAG VARIANT [VARIANT ...]   (env GAIT / N / LITERAL pass through)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2 3; do
  for b in ${BATCHES:-4096 1024 8192}; do
    timeout -k 10 120 python tools/perf_kernel.py default $b 20 >> $out/ab.txt 2>&1 || exit 1
    for v in "$@"; do
      QLOCO_LIB=tools/_var/$v/libqloco.so timeout -k 10 120 python tools/perf_kernel.py default $b 20 >> $out/ab.txt 2>&1 || exit 1
    done
  done
done
grep -v amdgpu.ids $out/ab.txt
