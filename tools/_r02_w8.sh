#!/bin/bash
# k_rollout_u at 8 waves/EU: rollout parity tests, then bench 2 / 3 / 4 streams interleaved (2 reps).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/w8
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -m gpu -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 1
for r in 1 2; do
  for s in 2 3 4; do
    timeout -k 10 120 python bench.py --streams $s --no-pmc --no-cpu-baseline >> $O/s$s.jsonl 2>> $O/err.log || exit 1
  done
done
