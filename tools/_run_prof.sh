set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 python tools/game_lengths.py 4096 > gpurun_out/lengths.json 2>&1 &&
timeout -k 10 120 python tools/game_lengths.py 65536 >> gpurun_out/lengths.json 2>&1
