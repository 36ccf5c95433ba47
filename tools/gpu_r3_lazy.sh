#!/bin/bash
# Lazy dual residuals at termination checks (P x skipped when the primal
# test fails) vs the full evaluation (tools/_var/nolazy,
# -DQLOCO_SRBD_LAZY_PX=0): GPU parity suite, then same-call A/B on the
# headline, small batches, configs 3-5 and the literal QP.
# Usage: tools/gpu_r3_lazy.sh TAG
set -o pipefail
tag=${1:-r3lz}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -n 1 $out/pytest_gpu.log
for rep in 1 2; do
  for w in "trot 10 4096 0" "trot 10 1 0" "trot 10 1024 0" "mixed 10 131072 0" "trot 16 65536 0" "pace 20 65536 0" "trot 10 4096 1"; do
    set -- $w
    for L in "" tools/_var/nolazy/libqloco.so; do
      tagl=lazy; [ -n "$L" ] && tagl=full
      GAIT=$1 N=$2 LITERAL=$4 QLOCO_LIB=$L timeout -k 10 180 python tools/perf_kernel.py default $3 10 2>&1 | grep -v amdgpu.ids | sed "s/^prod /$tagl/" >> $out/ab.txt || { tail -5 $out/ab.txt; exit 1; }
    done
  done
done
cat $out/ab.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
