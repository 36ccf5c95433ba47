#!/bin/bash
# Two-wave kernel evidence (verdict items 5 / literal line): ablation timings
# and SQ counter passes on the mixed config-5 share (N = 10 mixed, 131072)
# and the literal N = 10 trot batch (4096).  Usage: tools/gpu_r3_w2.sh TAG
set -o pipefail
tag=${1:-r3w2}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in default iter0 iter150; do
  GAIT=mixed timeout -k 10 120 python tools/perf_kernel.py $v 131072 5 >> $out/ablate.txt 2>&1 || exit 1
  LITERAL=1 timeout -k 10 120 python tools/perf_kernel.py $v 4096 10 >> $out/ablate.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $out/ablate.txt
for w in "mixed 131072 0" "trot 4096 1"; do
  set -- $w
  tg=$1$3
  GAIT=$1 LITERAL=$3 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $out/pmc1_$tg -o run -- python tools/perf_kernel.py default $2 2 > $out/pmc1_$tg.log 2>&1 || { tail -5 $out/pmc1_$tg.log; exit 1; }
  GAIT=$1 LITERAL=$3 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $out/pmc2_$tg -o run -- python tools/perf_kernel.py default $2 2 > $out/pmc2_$tg.log 2>&1 || { tail -5 $out/pmc2_$tg.log; exit 1; }
  echo "== $w" >> $out/pmc_sq.txt
  python tools/pmc_summary.py $out/pmc1_$tg srbd_admm_kernel >> $out/pmc_sq.txt && python tools/pmc_summary.py $out/pmc2_$tg srbd_admm_kernel >> $out/pmc_sq.txt
  rm -rf $out/pmc1_$tg $out/pmc2_$tg
done
cat $out/pmc_sq.txt
