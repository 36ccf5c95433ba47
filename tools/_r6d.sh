#!/bin/bash
set -o pipefail
out=gpurun_out/r6d; mkdir -p $out; cd "$GRAFT_REPO_ROOT" || exit 1
run() { timeout -k 10 300 python tools/lit_iters_ab.py "$@" >> $out/ab.txt 2>&1 || { tail -20 $out/ab.txt; exit 1; }; }
for n in 10 11 12 14 16; do run $n 48 trot isaac; done
export QLOCO_LIB=tools/_var/r5/libqloco.so
run 16 16 trot isaac
run 10 32 trot isaac
unset QLOCO_LIB
run 16 32 trot hardware
run 16 32 trot gazebo
grep -v amdgpu.ids $out/ab.txt | grep "B="
timeout -k 10 600 python -u -m pytest tests/test_qp_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest_qp.log 2>&1 || { tail -30 $out/pytest_qp.log; exit 1; }
tail -2 $out/pytest_qp.log
