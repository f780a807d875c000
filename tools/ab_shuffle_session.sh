# Batched shuffle (CIT_SHUFFLE_BATCH) on the GPU box: its bit-exact check
# against the serial draws, the cycle microbenchmark, then interleaved A/B of
# the main library (batched) against serial builds of the search unit
# (configs 3 / 4 / 4@512) and of the rollout unit (config 2).
#   bash tools/ab_shuffle_session.sh OUT
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_shuffle.py -x -q --timeout 120 --timeout-method thread > $O/test_shuffle.txt 2>&1 || exit 1
timeout -k 10 120 python tools/bench_shuffle.py > $O/bench_shuffle.jsonl 2>&1 || exit 1
M=citadels_self_play_amd/libcitadels_hip.so
for rep in 1 2; do
for lib in build/abshuf/libcfrbase.so $M; do
  v=$(basename $lib .so)
  CIT_LIB_PATH=$lib timeout -k 10 120 python tools/bench_cfr.py --batch 1024 --node-cap 4096 --reps 3 > $O/${v}_c3_$rep.log 2>&1 || exit 1
  CIT_LIB_PATH=$lib timeout -k 10 120 python tools/bench_cfr.py --pred --batch 512 --node-cap 4096 --reps 3 > $O/${v}_c4s_$rep.log 2>&1 || exit 1
  CIT_LIB_PATH=$lib timeout -k 10 120 python tools/bench_cfr.py --pred --batch 4096 --node-cap 4096 --reps 3 > $O/${v}_c4_$rep.log 2>&1 || exit 1
done
done
if [ -z "$AB_QUICK" ]; then
for rep in 1 2; do
for lib in build/abshuf/librollbase.so $M; do
  timeout -k 10 150 python tools/_ablib.py $lib 4096 > $O/roll_$(basename $lib .so)_$rep.json 2> $O/roll_$(basename $lib .so)_$rep.err || exit 1
done
done
fi
[ -n "$AB_QUICK" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_cfr.txt 2>&1 || exit 1
