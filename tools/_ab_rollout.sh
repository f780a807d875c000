#!/bin/bash
# A/B rollout builds: each lib benchmarked 3 times, interleaved (bench.py value lines).
set -o pipefail
mkdir -p gpurun_out/ab
for rep in 1 2 3; do
  for v in "$@"; do
    timeout -k 10 120 python tools/_ablib.py $v 4096 > gpurun_out/ab/$(basename $v .so)_$rep.log 2>&1 || exit 1
  done
done
for v in "$@"; do
  echo "$(basename $v .so) $(for rep in 1 2 3; do tail -1 gpurun_out/ab/$(basename $v .so)_$rep.log | python3 -c 'import json,sys; print(round(json.loads(sys.stdin.read())["value"]/1e6,1))'; done | tr '\n' ' ')"
done > gpurun_out/ab/summary.txt
