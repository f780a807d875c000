set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 &&
timeout -k 10 1000 bash tools/profile_gpu.sh > gpurun_out/prof.log 2>&1
