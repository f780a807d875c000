#!/bin/bash
# GPU check of the tree queue: parity tests, then config 5 batch vs queue.
set -o pipefail
O=gpurun_out/queue
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py tests/test_gpu_targets.py tests/test_gpu_dist.py -x -v --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_selfplay.py --config 5 --reps 1 --queue 2048 --batch 1024 --slice 0.1 > $O/c5q.json 2> $O/c5q.err &&
timeout -k 10 600 python -u tools/bench_selfplay.py --config 5 --iters 200000 --batch 320 --queue 960 --slice 0.5 --reps 1 --warmup 0 > $O/c5q_200k.json 2> $O/c5q_200k.err
