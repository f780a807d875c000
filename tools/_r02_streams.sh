#!/bin/bash
# bench.py --streams A/B (streams warmed before the timed region): 1 / 2 / 4 / 8 streams interleaved, 3 reps.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/streams2
mkdir -p $O
for r in 1 2 3; do
  for s in 1 2 4 8; do
    timeout -k 10 120 python bench.py --streams $s --no-pmc --no-cpu-baseline >> $O/s$s.jsonl 2>> $O/err.log || exit 1
    echo "rep $r streams $s done"
  done
done
timeout -k 10 120 python bench.py --streams 4 --steps 20 --no-pmc --no-cpu-baseline >> $O/s4_k20.jsonl 2>> $O/err.log &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k streams > $O/test.log 2>&1
