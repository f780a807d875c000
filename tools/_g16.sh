set -o pipefail
export TMPDIR=/tmp
for v in 0 32 64; do
  for b in 4096 16384; do
    timeout -k 10 120 python tools/_ablib.py build/libbuf$v.so $b > gpurun_out/ab_${v}_${b}.log 2>&1 || exit 1
  done
done
