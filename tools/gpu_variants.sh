#!/bin/bash
# time the product library and experimental variants: tools/gpu_variants.sh OUT VAR...
set -o pipefail
out=$1; shift
mkdir -p $(dirname $out)
timeout -k 10 300 python -m pytest tests/test_srbd_gpu.py -x -q -m gpu > ${out}.pytest 2>&1 || { tail -30 ${out}.pytest; exit 1; }
for B in 4096 8192; do for v in iter1 default; do
  timeout -k 10 60 python tools/perf_kernel.py $v $B 20 >> $out 2>&1 || exit 1
  for var in "$@"; do QLOCO_LIB=tools/_var/$var/libqloco.so timeout -k 10 60 python tools/perf_kernel.py $v $B 20 >> $out 2>&1 || exit 1; done
done; done
tail -1 ${out}.pytest; grep -v amdgpu.ids $out
