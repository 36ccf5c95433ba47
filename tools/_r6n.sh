#!/bin/bash
# round-6 measurement pass: A/B vs round 5, headline-only kernel trace,
# config-shape traffic and SQ counters, config lines, default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r6n; mkdir -p $out
for lib in cur r5 cur r5; do
  if [ $lib = cur ]; then unset QLOCO_LIB; else export QLOCO_LIB=tools/_var/r5/libqloco.so; fi
  timeout -k 10 120 python bench.py --steps 100 --warmup 5 --no-second-line --no-cpu-baseline > $out/ab.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$out/ab.json')); print('$lib', d['kernel_us_avg'], d['ms_per_step'])" | tee -a $out/ab.txt
done
unset QLOCO_LIB
bash tools/gpu.sh r6n ktraceh || exit 1
LITERAL=1 bash tools/gpu.sh r6n sq traffic || exit 1
N=16 GAIT=trot LITERAL=1 TB=65536 bash tools/gpu.sh r6n traffic || exit 1
N=20 GAIT=pace LITERAL=1 TB=65536 bash tools/gpu.sh r6n traffic || exit 1
N=10 GAIT=mixed LITERAL=1 TB=131072 bash tools/gpu.sh r6n traffic || exit 1
N=16 GAIT=trot LITERAL=1 TB=4096 bash tools/gpu.sh r6n sq || exit 1
N=20 GAIT=pace LITERAL=1 TB=4096 bash tools/gpu.sh r6n sq || exit 1
bash tools/gpu.sh r6n configs bench || exit 1
