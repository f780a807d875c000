#!/bin/bash
# bench.py 2 vs 3 streams (interleaved, 3 reps) and the N=2 folded gloo rehearsal with the default 2 streams.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/streams3
mkdir -p $O
for r in 1 2 3; do
  for s in 2 3; do
    timeout -k 10 120 python bench.py --streams $s --no-pmc --no-cpu-baseline >> $O/s$s.jsonl 2>> $O/err.log || exit 1
  done
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 4 --warmup 1 --dist-backend gloo --no-pmc > $O/dist_bench.json 2> $O/dist_bench.err
