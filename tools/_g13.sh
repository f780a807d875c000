set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python tools/_finderr.py 65536 32 > gpurun_out/finderr.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_jd.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --batch 16384 > gpurun_out/bench_jd16.log 2>&1
