set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/t_par.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_v2.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --batch 16384 > gpurun_out/bench_v2_16k.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --batch 16384 --games-per-block 1 > gpurun_out/bench_v2_16k_g1.log 2>&1
