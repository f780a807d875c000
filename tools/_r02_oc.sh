#!/bin/bash
# Overcommitted tree queue: GPU queue tests, then config 5 at cfr_train(200000).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/oc
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python tools/bench_selfplay.py --config 5 --iters 200000 --reps 1 --warmup 0 > $O/c5_oc2.json 2> $O/c5_oc2.err &&
timeout -k 10 300 python tools/bench_selfplay.py --config 5 --iters 200000 --reps 1 --warmup 0 --overcommit 3 > $O/c5_oc3.json 2> $O/c5_oc3.err
