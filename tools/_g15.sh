set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_cfr.py tests/test_gpu_mlp.py tests/test_gpu_targets.py tests/test_gpu_compare.py tests/test_gpu_api.py -x -q > gpurun_out/t_cfr.log 2>&1 &&
timeout -k 10 300 python tools/bench_selfplay.py --config 3 > gpurun_out/bs3.log 2>&1 &&
timeout -k 10 300 python tools/bench_selfplay.py --config 4 > gpurun_out/bs4.log 2>&1 &&
timeout -k 10 300 python tools/bench_selfplay.py --config 5 --iters 2000 --batch 1024 > gpurun_out/bs5a.log 2>&1 &&
timeout -k 10 300 python tools/_cfrprof.py > gpurun_out/cfrprof.log 2>&1
