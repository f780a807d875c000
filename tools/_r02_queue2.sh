#!/bin/bash
# Tree queue after the pruned target walk: parity, kernel split, config 5 batch vs queue.
set -o pipefail
O=gpurun_out/queue2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py tests/test_gpu_targets.py tests/test_gpu_dist.py tests/test_gpu_cfr.py -x -v --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o c5 -- python3 -u tools/bench_selfplay.py --config 5 --reps 1 --warmup 0 > $O/c5.json 2> $O/c5.err &&
timeout -k 10 200 python -u tools/bench_selfplay.py --config 5 --reps 1 --queue 2048 --batch 1024 --slice 0.1 > $O/c5q.json 2> $O/c5q.err &&
timeout -k 10 600 python -u tools/bench_selfplay.py --config 5 --iters 200000 --batch 320 --queue 960 --slice 0.5 --reps 1 --warmup 0 > $O/c5q_200k.json 2> $O/c5q_200k.err
