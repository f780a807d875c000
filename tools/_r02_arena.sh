#!/bin/bash
# GPU check of the block-allocated node pools: GPU suite, configs 3/4/5, config 5 at 200k with 320 trees.
set -o pipefail
O=gpurun_out/arena
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_selfplay.py --config 3 > $O/c3.json 2> $O/c3.err &&
timeout -k 10 200 python -u tools/bench_selfplay.py --config 4 > $O/c4.json 2> $O/c4.err &&
timeout -k 10 300 python -u tools/bench_selfplay.py --config 5 --reps 1 > $O/c5.json 2> $O/c5.err &&
timeout -k 10 500 python -u tools/bench_selfplay.py --config 5 --iters 200000 --batch 320 --reps 1 --warmup 0 > $O/c5_200k_320.json 2> $O/c5_200k_320.err
