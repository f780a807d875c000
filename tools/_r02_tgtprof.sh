#!/bin/bash
# Kernel split of config 5 (batch path): search vs target extraction.
set -o pipefail
O=gpurun_out/tgtprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c5 -o c5 -- python3 -u tools/bench_selfplay.py --config 5 --reps 1 --warmup 0 > $O/c5.json 2> $O/c5.err
