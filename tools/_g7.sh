set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_entry.py -x -q > gpurun_out/t_entry.log 2>&1
