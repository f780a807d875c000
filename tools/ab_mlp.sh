# A/B of leaf-MLP builds on the GPU box: the single-row wave forward latency
# (tools/bench_mlp.py --wave-only) and configs 4 / 4@512 with each library.
#   bash tools/ab_mlp.sh OUT LIB1 LIB2 ...
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
for lib in "$@"; do
  v=$(basename $lib .so)
  CIT_LIB_PATH=$lib timeout -k 10 120 python tools/bench_mlp.py --wave-only > $O/${v}_wave.jsonl 2>&1 || exit 1
done
for rep in 1 2; do
for lib in "$@"; do
  v=$(basename $lib .so)
  CIT_LIB_PATH=$lib timeout -k 10 120 python tools/bench_cfr.py --pred --batch 512 --node-cap 4096 --reps 3 > $O/${v}_c4s_$rep.log 2>&1 || exit 1
  CIT_LIB_PATH=$lib timeout -k 10 120 python tools/bench_cfr.py --pred --batch 4096 --node-cap 4096 --reps 3 > $O/${v}_c4_$rep.log 2>&1 || exit 1
done
done
