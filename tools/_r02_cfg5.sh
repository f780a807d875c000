#!/bin/bash
set -o pipefail
O=gpurun_out/cfg5
mkdir -p $O
DIAG_LIB=build/cfrdiag/libcfrdiag.so timeout -k 10 200 python -u tools/diag_cfr_errors.py 2000 1024 > $O/diag2000.json 2> $O/diag2000.err &&
DIAG_LIB=build/cfrdiag/libcfrdiag.so timeout -k 10 300 python -u tools/diag_cfr_errors.py 200000 64 > $O/diag200k.json 2> $O/diag200k.err &&
timeout -k 10 400 python -u tools/bench_selfplay.py --config 5 --iters 200000 --batch 160 --reps 1 --warmup 0 > $O/c5_200k_160.json 2> $O/c5_200k_160.err
