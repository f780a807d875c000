set -o pipefail
export TMPDIR=/tmp
CIT_ROLLOUT_VARIANT=4 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/t_par_u.log 2>&1 || exit 1
for v in 0 4; do
  for b in 4096 16384; do
    CIT_ROLLOUT_VARIANT=$v timeout -k 10 120 python bench.py --no-cpu-baseline --batch $b --games-per-block 1 --steps 5 > gpurun_out/var_${v}_${b}.log 2>&1 || exit 1
  done
done
