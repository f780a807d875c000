set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_selfplay.py --config 3 > gpurun_out/bs3.log 2>&1 &&
timeout -k 10 300 python tools/bench_selfplay.py --config 4 > gpurun_out/bs4.log 2>&1 &&
timeout -k 10 300 python tools/bench_selfplay.py --config 5 --iters 2000 --batch 1024 > gpurun_out/bs5a.log 2>&1 &&
timeout -k 10 600 python tools/bench_selfplay.py --config 5 --iters 20000 --batch 256 --reps 1 > gpurun_out/bs5b.log 2>&1
