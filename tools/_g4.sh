set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_api.py tests/test_gpu_targets.py -x -q > gpurun_out/t_api.log 2>&1
