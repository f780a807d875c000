set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_mlp.py -x -q > gpurun_out/t_mlp.log 2>&1 &&
timeout -k 10 300 python tools/bench_cfr.py --pred --batch 4096 --reps 2 > gpurun_out/c4.log 2>&1 &&
timeout -k 10 300 python tools/bench_cfr.py --pred --batch 16 --reps 1 >> gpurun_out/c4.log 2>&1
