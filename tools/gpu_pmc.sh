#!/bin/bash
# PMC counter passes for the SRBD kernel: tools/gpu_pmc.sh OUTDIR VARIANT...
set -o pipefail
out=$1; shift
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $out/pmc1_$v -o run -- python tools/perf_kernel.py $v 4096 3 > $out/pmc1_$v.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $out/pmc2_$v -o run -- python tools/perf_kernel.py $v 4096 3 > $out/pmc2_$v.log 2>&1 || exit 1
done
