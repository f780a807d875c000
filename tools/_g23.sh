set -o pipefail
export TMPDIR=/tmp
for v in base twistni os o2 o1 os_tni o2_tni; do
  timeout -k 10 120 python tools/_ablib.py build/ab/lib$v.so 4096 > gpurun_out/ab_$v.log 2>&1 || exit 1
done
