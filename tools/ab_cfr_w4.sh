set -o pipefail
O=gpurun_out/r05o; mkdir -p $O
for rep in 1 2; do
for v in cfrw3 cfrw4; do
  CIT_LIB_PATH=build/ab/lib$v.so timeout -k 10 120 python tools/bench_cfr.py --pred --batch 4096 --node-cap 4096 --reps 3 > $O/${v}_c4_$rep.log 2>&1 || exit 1
  CIT_LIB_PATH=build/ab/lib$v.so timeout -k 10 120 python tools/bench_cfr.py --batch 1024 --node-cap 4096 --reps 3 > $O/${v}_c3_$rep.log 2>&1 || exit 1
done
done
