set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1000 python -m pytest tests -m gpu -x -q > gpurun_out/t_gpu_all.log 2>&1
