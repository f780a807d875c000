#!/bin/bash
# Node creation stops listing at two options: CFR GPU tests, configs 3 / 4; then rollout unroll A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/u2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_cfr.py tests/test_gpu_targets.py tests/test_gpu_queue.py tests/test_gpu_api.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 200 python tools/bench_selfplay.py --config 3 --reps 5 > $O/c3.json 2> $O/c3.err &&
timeout -k 10 300 python tools/bench_selfplay.py --config 4 --reps 3 > $O/c4.json 2> $O/c4.err &&
bash tools/_r02_ab.sh 2 build/abr2/libbase.so build/abr2/libu1.so build/abr2/libu2.so build/abr2/libu3.so build/abr2/libu4.so
