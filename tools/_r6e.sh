#!/bin/bash
set -o pipefail
out=gpurun_out/r6e; mkdir -p $out; cd "$GRAFT_REPO_ROOT" || exit 1
run() { timeout -k 10 300 python tools/lit_iters_ab.py "$@" >> $out/ab.txt 2>&1 || { tail -20 $out/ab.txt; exit 1; }; }
run 16 48 trot isaac_iso
run 16 48 trot isaac_r7
export QLOCO_LIB=tools/_var/r5/libqloco.so
run 16 48 trot isaac_iso
run 16 48 trot isaac_r7
grep -v amdgpu.ids $out/ab.txt
