#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r6t; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_srbd_gpu.py -x -v -s --timeout 200 --timeout-method thread -k "reduced_iterate" > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
grep -E "max prim_res|passed|failed" $out/pytest.log
timeout -k 10 900 python -u tools/srbd_parity_scan.py 10 512 trot 1e-3 10 256 mixed 1e-3 16 128 trot 1e-3 20 96 pace 1e-3 20 64 mixed 1e-3 > $out/scan.txt 2>&1 || { tail -20 $out/scan.txt; exit 1; }
grep -v amdgpu.ids $out/scan.txt | grep -E "==|wrench|dF_adm|dM_adm|dX_adm|du0_adm"
