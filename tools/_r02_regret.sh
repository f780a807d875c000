#!/bin/bash
set -o pipefail
O=gpurun_out/regret
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_cfr.py tests/test_gpu_targets.py tests/test_gpu_queue.py tests/test_gpu_mlp.py -x -v --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_selfplay.py --config 3 --reps 5 > $O/c3.json 2> $O/c3.err &&
timeout -k 10 250 python -u tools/prof_cfr.py run top 200000:64 > $O/top.jsonl 2> $O/top.err
