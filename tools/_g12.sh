set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1000 python -m pytest tests -m gpu -x -q > gpurun_out/t_gpu_all.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench_u.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --batch 16384 > gpurun_out/bench_u16.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --batch 65536 --steps 3 > gpurun_out/bench_u64.log 2>&1
