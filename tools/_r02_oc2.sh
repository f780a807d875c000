#!/bin/bash
# Overcommit sweep for config 5 at cfr_train(200000): 960 trees at 1.5 / 2.5, 1920 trees at 1 / 2.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/oc2
mkdir -p $O
B="python tools/bench_selfplay.py --config 5 --iters 200000 --reps 1 --warmup 0"
timeout -k 10 200 $B --overcommit 1.5 > $O/q960_oc15.json 2> $O/q960_oc15.err &&
timeout -k 10 200 $B --overcommit 2.5 > $O/q960_oc25.json 2> $O/q960_oc25.err &&
timeout -k 10 300 $B --queue 1920 --overcommit 2 > $O/q1920_oc2.json 2> $O/q1920_oc2.err &&
timeout -k 10 300 $B --queue 1920 --overcommit 1 > $O/q1920_oc1.json 2> $O/q1920_oc1.err
