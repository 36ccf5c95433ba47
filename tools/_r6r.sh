#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r6r; mkdir -p $out
for lib in cur pre cur pre; do
  if [ $lib = cur ]; then unset QLOCO_LIB; else export QLOCO_LIB=tools/_var/pre_resume/libqloco.so; fi
  timeout -k 10 120 python bench.py --steps 100 --warmup 5 --no-second-line --no-cpu-baseline --lit-resume-cap -1 > $out/ab.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$out/ab.json')); print('$lib', d['kernel_us_avg'], d['ms_per_step'])" | tee -a $out/ab.txt
done
