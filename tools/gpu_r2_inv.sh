#!/bin/bash
# Product (DPP inverse, three-wave one-wave kernel) GPU suite; occupancy A/B
# (tools/_var/wpe2); MFMA-busy counters of the matrix-core inverse build
# (tools/_var/mfmainv) vs the product on N = 16 trot B = 65536.  Usage: TAG
set -o pipefail
tag=${1:-r2v}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -n 1 $out/pytest_gpu.log
for b in 1024 2048 4096 8192 65536; do
  timeout -k 10 120 python tools/perf_kernel.py default $b 10 >> $out/scan.txt 2>&1 || exit 1
  QLOCO_LIB=tools/_var/wpe2/libqloco.so timeout -k 10 120 python tools/perf_kernel.py default $b 10 >> $out/scan.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $out/scan.txt
for v in prod mfmainv; do
  envs="N=16"
  [ $v = mfmainv ] && envs="N=16 QLOCO_LIB=tools/_var/mfmainv/libqloco.so"
  env $envs timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $out/pmc_$v -o run -- python tools/perf_kernel.py default 65536 2 > $out/pmc_$v.log 2>&1 || { tail -20 $out/pmc_$v.log; exit 1; }
done
