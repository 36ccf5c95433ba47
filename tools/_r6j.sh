#!/bin/bash
set -o pipefail
out=gpurun_out/r6j; mkdir -p $out; cd "$GRAFT_REPO_ROOT" || exit 1
for v in default iter0 iter150 default; do
  for lib in cur r5; do
    if [ $lib = cur ]; then unset QLOCO_LIB; else export QLOCO_LIB=tools/_var/r5/libqloco.so; fi
    LITERAL=1 timeout -k 10 120 python tools/perf_kernel.py $v 4096 40 2>&1 | grep -v amdgpu.ids | sed "s|^|$lib |" >> $out/ab.txt || exit 1
  done
done
cat $out/ab.txt
