#!/bin/bash
# A/B of the Gauss-Jordan forms (QLOCO_GJ_MODE 0 / 1 / 2, variant libraries
# gj0 gj1 gj2) on the parity envelopes: tight eps reduced, default eps mixed,
# literal tight and default.  Usage: tools/gpu_gjmode.sh TAG
set -o pipefail
tag=${1:-gjmode}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in ${GJV:-0 1 2}; do
  QLOCO_LIB=tools/_var/$m/libqloco.so timeout -k 10 300 python -u tools/srbd_parity_scan.py 10 32 trot 1e-6 20 12 pace 1e-6 20 8 mixed 1e-6 10 24 mixed 1e-6 10 48 mixed 1e-3 >> $out/scan.txt 2>&1 || exit 1
  QLOCO_LIB=tools/_var/$m/libqloco.so timeout -k 10 300 python -u tools/srbd_parity_scan.py --literal 10 24 trot 1e-6 10 48 pace 1e-3 >> $out/scan.txt 2>&1 || exit 1
done
grep -E "==|wrench|dX_adm|dX_ex |gap_gpu" $out/scan.txt
