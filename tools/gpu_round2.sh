set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_srbd_gpu.py tests/test_qp_gpu.py -q > gpurun_out/pytest_gpu2.log 2>&1
echo "pytest exit=$?" >> gpurun_out/pytest_gpu2.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof2.log 2>&1
echo "bench/prof exit=$?" >> gpurun_out/bench2.log
