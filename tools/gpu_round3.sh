#!/bin/bash
# GPU check after the SRBD kernel restructure: parity tests, ablation, bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_srbd_gpu.py -x -q -m gpu > gpurun_out/pytest_srbd3.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_srbd3.log; exit 1; }
timeout -k 10 200 python tools/perf_ablate.py > gpurun_out/ablate3.log 2>&1 || { echo "ablate failed"; tail -20 gpurun_out/ablate3.log; exit 1; }
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-seconds 5 > gpurun_out/bench3.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench3.log; exit 1; }
tail -3 gpurun_out/pytest_srbd3.log; cat gpurun_out/ablate3.log; cat gpurun_out/bench3.log
