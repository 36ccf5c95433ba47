#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r6s; mkdir -p $out
for spec in "10 4096 trot" "10 4096 mixed" "7 2048 pace"; do
  set -- $spec
  timeout -k 10 120 python tools/lit_dump_out.py $out/cur.npz $1 $2 $3 || exit 1
  QLOCO_LIB=tools/_var/pkmv/libqloco.so timeout -k 10 120 python tools/lit_dump_out.py $out/pk.npz $1 $2 $3 || exit 1
  python -c "
import numpy as np; a=np.load('$out/cur.npz'); b=np.load('$out/pk.npz')
print('$spec', {k: bool(np.array_equal(a[k].view(np.int32) if a[k].dtype==np.float32 else a[k], b[k].view(np.int32) if b[k].dtype==np.float32 else b[k])) for k in a.files})" | tee -a $out/ab.txt
done
for lib in cur pk cur pk; do
  if [ $lib = cur ]; then unset QLOCO_LIB; else export QLOCO_LIB=tools/_var/pkmv/libqloco.so; fi
  timeout -k 10 120 python bench.py --steps 100 --warmup 5 --no-second-line --no-cpu-baseline > $out/b.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$out/b.json')); print('$lib', d['kernel_us_avg'], d['ms_per_step'])" | tee -a $out/ab.txt
done
