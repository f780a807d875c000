set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_selfplay.py --config 5 --reps 1 --batch 512 --node-cap 100000 --edge-cap 300000 > gpurun_out/cfg5_512.log 2>&1 &&
timeout -k 10 300 python tools/bench_selfplay.py --config 5 --reps 1 --batch 1024 --node-cap 100000 --edge-cap 250000 > gpurun_out/cfg5_1024.log 2>&1
