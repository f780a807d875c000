#!/bin/bash
# Interleaved A/B of rollout builds: bash tools/_r02_ab.sh REPS lib1.so lib2.so ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
R=$1; shift
for r in $(seq 1 $R); do
  for v in "$@"; do
    timeout -k 10 120 python tools/_ablib.py $v 4096 > $O/$(basename $v .so)_$r.json 2> $O/$(basename $v .so)_$r.err || exit 1
  done
done
