#!/bin/bash
# Two-wave buckets back at three waves/SIMD (no in-loop spills): GPU parity
# suite, same-call A/B on the mixed config-5 share against the four-wave
# build (tools/_var/w2w4), HBM traffic of the shipped buckets, smoke, the
# headline bench line and the config-5 line.  Usage: tools/gpu_r3_w2_final.sh TAG
set -o pipefail
tag=${1:-r3wf}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -n 1 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
for rep in 1 2; do
  for L in "" tools/_var/w2w4/libqloco.so; do
    tagl=w3; [ -n "$L" ] && tagl=w4
    GAIT=mixed N=10 QLOCO_LIB=$L timeout -k 10 180 python tools/perf_kernel.py default 131072 5 2>&1 | grep -v amdgpu.ids | sed "s/^prod /$tagl  /" >> $out/ab.txt || { tail -5 $out/ab.txt; exit 1; }
  done
done
cat $out/ab.txt
for ctr in FETCH_SIZE WRITE_SIZE; do
  GAIT=mixed N=10 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d $out/$ctr -o run -- python tools/perf_kernel.py default 131072 2 > $out/$ctr.log 2>&1 || { tail -20 $out/$ctr.log; exit 1; }
done
for k in "2, 3, false, 20, 3>" "2, 3, false, 20, 6>" "1, 3, false, 20, 16>"; do
  echo "kernel <$k" >> $out/traffic.txt
  python tools/prof_summary.py traffic $out/FETCH_SIZE $out/WRITE_SIZE "$k" $out/tmp.json 2>&1 | tr -d '\n' >> $out/traffic.txt
  echo >> $out/traffic.txt
done
rm -rf $out/FETCH_SIZE $out/WRITE_SIZE
cat $out/traffic.txt
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 240 python bench.py --horizon 10 --gait mixed --batch 131072 --steps 20 --warmup 3 --no-cpu-baseline > $out/config5.json 2> $out/config5.err || { tail -20 $out/config5.err; exit 1; }
cat $out/config5.json
