#!/bin/bash
set -o pipefail
out=${1:-gpurun_out/mfma.log}
mkdir -p $(dirname $out)
timeout -k 10 60 ./tools/micro/mfma4x4 >> $out 2>&1 || exit 1
timeout -k 10 400 python -m pytest tests/test_srbd_gpu.py tests/test_host_gpu.py -m gpu -x -q >> $out 2>&1 || exit 1
bash tools/gpu_variants.sh $out "gjdpp" "1024 4096 8192" || exit 1
bash tools/gpu_variants.sh $out "gjdpp" "8192" 16 trot || exit 1
