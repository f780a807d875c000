# A/B of search builds on the GPU box: configs 3 (1,024 trees), 4 (4,096)
# and 4@512 with each library, interleaved, 2 rounds of 3 reps.
#   bash tools/ab_cfr.sh OUT LIB1 LIB2 ...     (LIBs: paths of libcitadels_hip.so builds)
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
for rep in 1 2; do
for lib in "$@"; do
  v=$(basename $lib .so)
  CIT_LIB_PATH=$lib timeout -k 10 120 python tools/bench_cfr.py --batch 1024 --node-cap 4096 --reps 3 > $O/${v}_c3_$rep.log 2>&1 || exit 1
  CIT_LIB_PATH=$lib timeout -k 10 120 python tools/bench_cfr.py --pred --batch 512 --node-cap 4096 --reps 3 > $O/${v}_c4s_$rep.log 2>&1 || exit 1
  CIT_LIB_PATH=$lib timeout -k 10 120 python tools/bench_cfr.py --pred --batch 4096 --node-cap 4096 --reps 3 > $O/${v}_c4_$rep.log 2>&1 || exit 1
done
done
