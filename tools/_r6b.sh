#!/bin/bash
# one-off A/B of literal iteration parity: current tree vs the round-5 kernels
set -o pipefail
out=gpurun_out/r6b; mkdir -p $out; cd "$GRAFT_REPO_ROOT" || exit 1
for spec in "20 64 mixed" "16 64 mixed" "20 32 pace" "13 32 trot"; do
  for lib in cur r5; do
    if [ $lib = cur ]; then unset QLOCO_LIB; else export QLOCO_LIB=tools/_var/r5/libqloco.so; fi
    timeout -k 10 300 python tools/lit_iters_ab.py $spec >> $out/ab.txt 2>&1 || { tail -20 $out/ab.txt; exit 1; }
  done
done
unset QLOCO_LIB
for spec in "10 32 trot isaac" "16 16 trot isaac" "20 12 pace isaac"; do
  timeout -k 10 300 python tools/lit_iters_ab.py $spec >> $out/ab.txt 2>&1 || { tail -20 $out/ab.txt; exit 1; }
done
grep -v amdgpu.ids $out/ab.txt
