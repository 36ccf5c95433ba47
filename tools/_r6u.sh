#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r6u; mkdir -p $out
timeout -k 10 900 python -u tools/srbd_parity_scan.py 10 512 trot 1e-3 10 256 mixed 1e-3 16 128 trot 1e-3 20 96 pace 1e-3 20 64 mixed 1e-3 > $out/scan.txt 2>&1 || { tail -20 $out/scan.txt; exit 1; }
grep -v amdgpu.ids $out/scan.txt | grep -E "==|wrench|du0 "
