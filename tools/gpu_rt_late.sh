#!/bin/bash
# rt tick time vs walking time (warm-up 150 / 1000 / 1500 ticks), product
# library against tools/_var/prev (build it with tools/variant_lib.py from
# the tree to compare against, and drop ./tools/_var from .gpurunignore for
# the call).
set -o pipefail
mkdir -p gpurun_out/late
for W in 150 1000 1500; do
  timeout -k 10 240 python tools/bench_rt.py --sets 10 --no-cpu-baseline --warmup $W > gpurun_out/late/new_$W.json 2>>gpurun_out/late/err || exit 1
  QLOCO_LIB=tools/_var/prev/libqloco.so timeout -k 10 240 python tools/bench_rt.py --sets 10 --no-cpu-baseline --warmup $W > gpurun_out/late/prev_$W.json 2>>gpurun_out/late/err || exit 1
done
for f in gpurun_out/late/*.json; do python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['ms_per_step']*1e3,1), d['body_mpc_ran_frac'])" $f; done
