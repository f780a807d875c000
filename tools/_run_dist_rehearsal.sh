#!/bin/bash
# N=2 rehearsal of the multi-rank paths on a one-GPU box: both ranks fold onto
# cuda:0 and talk over gloo (the real N>1 path is RCCL, one rank per GPU).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo > gpurun_out/dist_bench.json 2> gpurun_out/dist_bench.err &&
CIT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 \
  tools/bench_selfplay.py --config 5 --reps 1 --batch 64 --iters 2000 > gpurun_out/dist_cfg5.log 2>&1 &&
CIT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 \
  tools/bench_selfplay.py --config 4 --reps 1 --batch 256 > gpurun_out/dist_cfg4.log 2>&1
