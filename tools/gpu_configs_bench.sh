#!/bin/bash
# bench.py lines for BASELINE configs 2-5 on one GPU (per-GPU shares of the
# 8-GPU configs), plus a rocprofv3 kernel-trace of each.  Usage: tools/gpu_configs_bench.sh TAG
set -o pipefail
tag=${1:-cfg}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for spec in "16 trot 65536" "20 pace 65536" "10 mixed 131072"; do
  set -- $spec
  timeout -k 10 240 python bench.py --horizon $1 --gait $2 --batch $3 --steps 30 --warmup 3 --no-cpu-baseline >> $out/configs.jsonl 2>> $out/configs.err || { tail -20 $out/configs.err; exit 1; }
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/kt_$1_$2 -o run -- python bench.py --horizon $1 --gait $2 --batch $3 --steps 10 --warmup 2 --no-cpu-baseline > $out/kt_$1_$2.log 2>&1 || { tail -20 $out/kt_$1_$2.log; exit 1; }
done
cat $out/configs.jsonl
