#!/bin/bash
# W = 2 matrix-core inverse: GPU parity suite, then configs 3-5 per-GPU
# shares + the headline against the DPP Gauss-Jordan build (tools/_var/dppinv),
# rocprofv3 stats of the N = 16 config.  Usage: TAG
set -o pipefail
tag=${1:-r2w}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || true
tail -n 1 $out/pytest_gpu.log
for spec in "16 trot 65536" "20 pace 65536" "10 mixed 131072" "10 trot 4096"; do
  set -- $spec
  for mode in mfma dpp; do
    envs=""
    [ $mode = dpp ] && envs="QLOCO_LIB=tools/_var/dppinv/libqloco.so"
    env $envs timeout -k 10 240 python bench.py --horizon $1 --gait $2 --batch $3 --steps 20 --warmup 3 --no-cpu-baseline > $out/b_$1_$2_$mode.json 2>> $out/configs.err || { tail -20 $out/configs.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$out/b_$1_$2_$mode.json')); print('%-7s N=%-2s %-6s B=%-7s %8.3f ms/step %10.0f solves/s frac %.3f exec %.3f' % ('$mode', '$1', '$2', '$3', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['executed_frac']))" >> $out/configs.txt
  done
done
cat $out/configs.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/kt16 -o run -- python bench.py --horizon 16 --gait trot --batch 65536 --steps 5 --warmup 2 --no-cpu-baseline > $out/kt16.log 2>&1 || { tail -20 $out/kt16.log; exit 1; }
