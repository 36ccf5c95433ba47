#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r6o; mkdir -p $out
for a in "--ticks 1" "--ticks 8" "--ticks 8 --ungrouped" "--ticks 1 --ungrouped"; do
  timeout -k 10 200 python tools/bench_qp.py --no-cpu-baseline $a >> $out/bench_qp_ticks.jsonl 2>> $out/qp.err || { tail $out/qp.err; exit 1; }
done
python - <<'PY'
import json
for l in open("gpurun_out/r6o/bench_qp_ticks.jsonl"):
    d = json.loads(l); print(round(d["ms_per_step"], 4), d["config"]["workload"])
PY
bash tools/gpu.sh r6o sqqp bench || exit 1
