#!/bin/bash
# rt node tick: robots scan (occupancy) + SQ PMC pass per rt kernel at 65536
# robots.  Usage: tools/gpu_rt_perf.sh TAG
set -o pipefail
tag=${1:-rtperf}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for B in 65536 131072 262144; do
  timeout -k 10 240 python tools/bench_rt.py --robots $B --sets 10 --no-cpu-baseline >> $out/scan.jsonl 2>> $out/scan.err || { tail -20 $out/scan.err; exit 1; }
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/kt -o run -- python tools/bench_rt.py --sets 10 --no-cpu-baseline --steps 30 > $out/kt.log 2>&1 || { tail -20 $out/kt.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM -d $out/pmc1_rt -o run -- python tools/bench_rt.py --sets 10 --no-cpu-baseline --steps 10 > $out/pmc1.log 2>&1 || { tail -20 $out/pmc1.log; exit 1; }
python - "$out/scan.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["config"]["workload"], "%.3g" % d["value"], round(d["ms_per_step"] * 1e3, 1), "us", round(d["roofline"]["frac"], 3))
PY
python tools/prof_summary.py stats $out/kt $out/kt_stats.csv | head -5
for k in rt_pre rt_post body_mpc; do python tools/pmc_summary.py $out $k; done
