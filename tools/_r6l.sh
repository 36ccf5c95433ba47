#!/bin/bash
set -o pipefail
out=gpurun_out/r6l; mkdir -p $out; cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u tools/srbd_parity_scan.py --literal 20 128 mixed 1e-3 16 128 mixed 1e-3 15 64 mixed 1e-3 > $out/scan.txt 2>&1 || { tail -20 $out/scan.txt; exit 1; }
grep -v amdgpu.ids $out/scan.txt | grep -E "==|wrench|du0|dit"
timeout -k 10 600 python -u -m pytest tests/test_srbd_gpu.py -x -v -s --timeout 200 --timeout-method thread -k "termination or reference_weight or edge_cases" > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
grep -E "max prim_res|passed|failed" $out/pytest.log
