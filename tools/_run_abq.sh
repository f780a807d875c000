set -o pipefail
export TMPDIR=/tmp
for v in "$@"; do
  timeout -k 10 120 python tools/_ablib.py $v 4096 > gpurun_out/ab_$(basename $v .so).log 2>&1 || exit 1
done
