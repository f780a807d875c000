set -o pipefail
export TMPDIR=/tmp
timeout -k 10 200 python tools/_dbg_close.py > gpurun_out/dbg.log 2>&1 &&
timeout -k 10 900 python -m pytest tests/test_gpu_api.py tests/test_gpu_targets.py -x -q > gpurun_out/t_api.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_nsa.log 2>&1
