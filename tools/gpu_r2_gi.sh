#!/bin/bash
# Phase clocks of the Goldfarb-Idnani core in force_qp_kernel + the force QP
# and rt-tick bench lines.  Usage: TAG
set -o pipefail
tag=${1:-r2g}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for b in 65536; do
  QLOCO_LIB=tools/_var/giphase/libqloco.so timeout -k 10 120 python tools/gi_phase.py $b >> $out/gi_phase.txt 2>&1 || { tail -20 $out/gi_phase.txt; exit 1; }
done
grep -v amdgpu.ids $out/gi_phase.txt
timeout -k 10 200 python tools/bench_qp.py --no-cpu-baseline > $out/bench_qp.json 2> $out/bench_qp.err || { tail -20 $out/bench_qp.err; exit 1; }
cat $out/bench_qp.json
