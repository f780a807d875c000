#!/bin/bash
# Configs 3-5 measurement on the GPU box (one process each, own time limit).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_selfplay.py --config 3 --reps 2 > gpurun_out/cfg3.log 2>&1 &&
timeout -k 10 300 python tools/bench_selfplay.py --config 4 --reps 2 > gpurun_out/cfg4.log 2>&1 &&
timeout -k 10 300 python tools/bench_selfplay.py --config 5 --reps 1 --batch 1024 --node-cap 100000 --edge-cap 250000 > gpurun_out/cfg5_1024.log 2>&1
