#!/bin/bash
# Split vs row one-wave kernel: setup / iteration ablations and SQ counters
# at B = 65536 (issue-bound) and 4096.  Usage: tools/gpu_r3_split2.sh TAG
set -o pipefail
tag=${1:-r3split2}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for b in 65536 4096; do
  for v in default iter0 iter150; do
    timeout -k 10 120 python tools/perf_kernel.py $v $b 5 >> $out/ablate.txt 2>&1 || exit 1
    QLOCO_LIB=tools/_var/row4/libqloco.so timeout -k 10 120 python tools/perf_kernel.py $v $b 5 >> $out/ablate.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $out/ablate.txt
for lib in prod row4; do
  L=""; [ $lib = row4 ] && L=tools/_var/row4/libqloco.so
  QLOCO_LIB=$L timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $out/pmc1_$lib -o run -- python tools/perf_kernel.py default 65536 2 > $out/pmc1_$lib.log 2>&1 || { tail -5 $out/pmc1_$lib.log; exit 1; }
  QLOCO_LIB=$L timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $out/pmc2_$lib -o run -- python tools/perf_kernel.py default 65536 2 > $out/pmc2_$lib.log 2>&1 || { tail -5 $out/pmc2_$lib.log; exit 1; }
  echo "== $lib 65536" >> $out/pmc_sq.txt
  python tools/pmc_summary.py $out/pmc1_$lib srbd_ >> $out/pmc_sq.txt && python tools/pmc_summary.py $out/pmc2_$lib srbd_ >> $out/pmc_sq.txt
  rm -rf $out/pmc1_$lib $out/pmc2_$lib
done
cat $out/pmc_sq.txt
