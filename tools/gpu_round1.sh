set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_srbd_gpu.py -x -q > gpurun_out/pytest_gpu1.log 2>&1
echo "pytest exit=$?" >> gpurun_out/pytest_gpu1.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof1.log 2>&1
echo "bench/prof exit=$?" >> gpurun_out/bench1.log
