set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 python tools/prof_rollout.py 4096 > gpurun_out/prof_rollout.json 2>&1
