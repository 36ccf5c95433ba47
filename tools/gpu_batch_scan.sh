#!/bin/bash
# Headline workload (Go1 trot N = 10) across batch sizes: bench.py lines
# (latency of a single robot's solve at B = 1 up to throughput at B = 65536).
# Usage: tools/gpu_batch_scan.sh TAG
set -o pipefail
tag=${1:-scan}
out=gpurun_out/$tag
mkdir -p $out
for B in 1 64 256 1024 2048 4096 8192 16384 65536; do
  timeout -k 10 180 python bench.py --batch $B --steps 100 --warmup 10 --no-cpu-baseline >> $out/scan.jsonl 2>> $out/scan.err || { tail -20 $out/scan.err; exit 1; }
done
python - "$out/scan.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["config"]["batch_per_gpu"], round(d["value"]), d["kernel_us_avg"], d["p99_batch_us"], d["roofline"]["frac"])
PY
