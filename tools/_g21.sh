set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cfr.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t21.log 2>&1 &&
timeout -k 10 120 python tools/prof_rollout.py 4096 > gpurun_out/prof_rollout.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench21.log 2>&1
