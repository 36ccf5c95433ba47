#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r6p; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_srbd_gpu.py -x -v -s --timeout 120 --timeout-method thread -k "capped_resume" > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
grep -E "resumed|passed|failed" $out/pytest.log
for cap in 0 -1 0 -1 100 150; do
  timeout -k 10 120 python bench.py --steps 100 --warmup 5 --no-second-line --no-cpu-baseline --lit-resume-cap $cap > $out/ab.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$out/ab.json')); print('cap $cap', d['kernel_us_avg'], d['ms_per_step'], d['roofline']['frac'])" | tee -a $out/ab.txt
done
