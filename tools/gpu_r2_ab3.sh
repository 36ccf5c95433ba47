#!/bin/bash
# Same-call A/B of the headline: session-start library vs the current tree
# (three-wave) vs the current tree built two-wave.  Usage: TAG
set -o pipefail
tag=${1:-r2ab}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
for lib in cur r2start; do
  envs=""
  [ $lib != cur ] && envs="QLOCO_LIB=tools/_var/$lib/libqloco.so"
  for b in 2048 4096 8192; do
    env $envs timeout -k 10 120 python tools/perf_kernel.py default $b 20 | sed "s/^[a-z0-9]* /$lib /" >> $out/ab.txt 2>&1 || exit 1
  done
  env $envs timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $out/ab_$lib.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$out/ab_$lib.json')); print('$lib bench', d['ms_per_step'], d['value'])" >> $out/ab.txt
done
done
grep -v amdgpu.ids $out/ab.txt
