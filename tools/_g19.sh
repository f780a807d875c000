set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 python tools/diag_rollout.py 4096 > gpurun_out/diag_rollout.log 2>&1 &&
timeout -k 10 120 python tools/diag_rollout.py 1024 >> gpurun_out/diag_rollout.log 2>&1 &&
timeout -k 10 300 python tools/diag_cfr_errors.py > gpurun_out/diag_cfr.log 2>&1
