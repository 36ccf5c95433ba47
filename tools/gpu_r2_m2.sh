#!/bin/bash
# Explicit-diagonal matrix-core inverse on the two-wave kernel only
# (tools/_var/mfma2w2): SRBD parity suite against it, then configs 3-5 and
# the headline vs the product.  Usage: TAG
set -o pipefail
tag=${1:-r2m2}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
QLOCO_LIB=tools/_var/mfma2w2/libqloco.so timeout -k 10 600 python -u -m pytest tests/test_srbd_gpu.py -m gpu -v --timeout 120 --timeout-method thread > $out/pytest_srbd.log 2>&1
tail -n 3 $out/pytest_srbd.log; grep FAILED $out/pytest_srbd.log
for spec in "16 trot 65536" "20 pace 65536" "10 mixed 131072" "10 trot 4096"; do
  set -- $spec
  for mode in prod mfma2w2; do
    envs=""
    [ $mode = mfma2w2 ] && envs="QLOCO_LIB=tools/_var/mfma2w2/libqloco.so"
    env $envs timeout -k 10 240 python bench.py --horizon $1 --gait $2 --batch $3 --steps 20 --warmup 3 --no-cpu-baseline > $out/b.json 2>> $out/configs.err || { tail -20 $out/configs.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$out/b.json')); print('%-8s N=%-2s %-6s B=%-7s %8.3f ms/step %10.0f solves/s frac %.3f exec %.3f' % ('$mode', '$1', '$2', '$3', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['executed_frac']))" >> $out/configs.txt
  done
done
cat $out/configs.txt
