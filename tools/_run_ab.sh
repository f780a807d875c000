set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_gpu_tests.log 2>&1 &&
for v in "$@"; do
  timeout -k 10 120 python tools/_ablib.py $v 4096 > gpurun_out/ab_$(basename $v .so).log 2>&1 || exit 1
done &&
timeout -k 10 200 python tools/bench_selfplay.py --config 3 > gpurun_out/cfg3.log 2>&1 &&
timeout -k 10 200 python tools/bench_selfplay.py --config 4 > gpurun_out/cfg4.log 2>&1 &&
timeout -k 10 300 python tools/bench_selfplay.py --config 5 --reps 1 > gpurun_out/cfg5.log 2>&1
