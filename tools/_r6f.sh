#!/bin/bash
set -o pipefail
out=gpurun_out/r6f; mkdir -p $out; cd "$GRAFT_REPO_ROOT" || exit 1
N=16 QSET=isaac INST=5,22,27 timeout -k 10 300 python tools/lit_debug.py 48 trot rho > $out/rho.txt 2>&1 || { tail -20 $out/rho.txt; exit 1; }
grep -v amdgpu.ids $out/rho.txt
