#!/bin/bash
# round-2 GPU check: full -m gpu suite, then a config-5 run at the reference's 200000 iterations
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 600 python -u tools/bench_selfplay.py --config 5 --iters 200000 --batch 64 --reps 1 --warmup 0 > gpurun_out/cfg5_200k.json 2> gpurun_out/cfg5_200k.err
