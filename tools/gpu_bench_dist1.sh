#!/bin/bash
# bench.py's multi-rank code path (RCCL group + all-gather, overlapped and not)
# on one GPU (torchrun, one rank, --force-dist), and the plain N = 1 line.
set -o pipefail
mkdir -p gpurun_out/dist1
export MASTER_ADDR=127.0.0.1
timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline > gpurun_out/dist1/n1.json 2> gpurun_out/dist1/n1.err || { tail -20 gpurun_out/dist1/n1.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --steps 100 --no-cpu-baseline --force-dist --overlap > gpurun_out/dist1/overlap.json 2> gpurun_out/dist1/overlap.err || { tail -20 gpurun_out/dist1/overlap.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29532 bench.py --steps 100 --no-cpu-baseline --force-dist > gpurun_out/dist1/serial.json 2> gpurun_out/dist1/serial.err || { tail -20 gpurun_out/dist1/serial.err; exit 1; }
for f in n1 overlap serial; do python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']), d['ms_per_step'], d['config']['parallelism'], d['status_ok_frac'])" gpurun_out/dist1/$f.json; done
