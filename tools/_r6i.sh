#!/bin/bash
set -o pipefail
out=gpurun_out/r6i; mkdir -p $out; cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for lib in cur r5; do
    if [ $lib = cur ]; then unset QLOCO_LIB; else export QLOCO_LIB=tools/_var/r5/libqloco.so; fi
    timeout -k 10 120 python bench.py --steps 100 --warmup 5 --no-second-line --no-cpu-baseline > $out/b_${lib}_$rep.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open('$out/b_${lib}_$rep.json')); print('$lib', $rep, d['kernel_us_avg'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
