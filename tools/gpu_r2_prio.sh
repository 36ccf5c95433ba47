#!/bin/bash
# s_setprio by iteration count (QLOCO_SRBD_PRIO variants) vs the product.
set -o pipefail
tag=${1:-r2p}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for b in 1024 4096 8192 65536; do
  timeout -k 10 120 python tools/perf_kernel.py default $b 10 >> $out/scan.txt 2>&1 || exit 1
  for v in prio50 prio100; do
    QLOCO_LIB=tools/_var/$v/libqloco.so timeout -k 10 120 python tools/perf_kernel.py default $b 10 >> $out/scan.txt 2>&1 || exit 1
  done
done
for spec in "16 trot 65536" "10 mixed 131072"; do
  set -- $spec
  for v in prod prio50; do
    envs="N=$1 GAIT=$2"
    [ $v = prio50 ] && envs="$envs QLOCO_LIB=tools/_var/prio50/libqloco.so"
    env $envs timeout -k 10 120 python tools/perf_kernel.py default $3 5 >> $out/scan.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $out/scan.txt
