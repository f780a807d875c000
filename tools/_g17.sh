set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -x -q > gpurun_out/t_par.log 2>&1 &&
timeout -k 10 400 python tools/_finderr.py 65536 16 > gpurun_out/finderr.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench_buf.log 2>&1
