#!/bin/bash
# Round-3 measurement of the shipped tree: GPU parity suite, smoke,
# headline bench line, rocprofv3 kernel stats, SQ counter passes and HBM
# traffic passes of the headline kernel, configs 3-5 lines, force-QP and
# rt-tick lines.  Usage: tools/gpu_r3_final.sh TAG (w3: the 3-waves/SIMD one-wave kernel)
set -o pipefail
tag=${1:-r3z}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -n 1 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/ktrace -o run -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $out/ktrace.log 2>&1 || { tail -20 $out/ktrace.log; exit 1; }
python tools/db_kernel_stats.py $out/ktrace > $out/kernel_stats.csv && rm -rf $out/ktrace
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $out/pmc1 -o run -- python tools/perf_kernel.py default 4096 3 > $out/pmc1.log 2>&1 || { tail -20 $out/pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $out/pmc2 -o run -- python tools/perf_kernel.py default 4096 3 > $out/pmc2.log 2>&1 || { tail -20 $out/pmc2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/fetch -o run -- python tools/perf_kernel.py default 4096 3 > $out/fetch.log 2>&1 || { tail -20 $out/fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $out/write -o run -- python tools/perf_kernel.py default 4096 3 > $out/write.log 2>&1 || { tail -20 $out/write.log; exit 1; }
python tools/pmc_summary.py $out/pmc1 srbd_admm > $out/pmc_sq.txt && python tools/pmc_summary.py $out/pmc2 srbd_admm >> $out/pmc_sq.txt
python tools/prof_summary.py traffic $out/fetch $out/write srbd_admm $out/traffic_srbd_n10_b4096.json > /dev/null
rm -rf $out/pmc1 $out/pmc2 $out/fetch $out/write
for lib in cur w3; do
  [ $lib = w3 ] && [ ! -f tools/_var/w3/libqloco.so ] && continue
  envs=""
  [ $lib = w3 ] && envs="QLOCO_LIB=tools/_var/w3/libqloco.so"
  env $envs timeout -k 10 120 python tools/perf_kernel.py default 4096 20 | sed "s/^[a-z0-9]* /$lib /" >> $out/ab_w3.txt 2>&1 || exit 1
  env $envs timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $out/ab_$lib.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$out/ab_$lib.json')); print('$lib bench', d['ms_per_step'], d['value'])" >> $out/ab_w3.txt
done
cat $out/ab_w3.txt
for spec in "16 trot 65536" "20 pace 65536" "10 mixed 131072"; do
  set -- $spec
  timeout -k 10 240 python bench.py --horizon $1 --gait $2 --batch $3 --steps 20 --warmup 3 --no-cpu-baseline >> $out/configs.jsonl 2>> $out/configs.err || { tail -20 $out/configs.err; exit 1; }
done
for b in 1 1024 2048 4096 8192 16384 65536; do
  timeout -k 10 120 python tools/perf_kernel.py default $b 10 >> $out/scan.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $out/scan.txt
timeout -k 10 200 python tools/bench_qp.py > $out/bench_qp.json 2> $out/bench_qp.err || { tail -20 $out/bench_qp.err; exit 1; }
timeout -k 10 200 python tools/bench_rt.py > $out/bench_rt.json 2> $out/bench_rt.err || { tail -20 $out/bench_rt.err; exit 1; }
cat $out/configs.jsonl $out/bench_qp.json $out/bench_rt.json
