set -o pipefail
O=gpurun_out/r04j; mkdir -p $O
CIT_LIB_PATH=build/abw4/libw4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_cfr.py tests/test_gpu_mlp.py tests/test_gpu_configs.py -x -q -k "not train_from_scratch" --timeout 200 --timeout-method thread > $O/tests_w4.txt 2>&1; echo "tests rc=$?" >> $O/status.txt
grep -q "failed\|error" $O/tests_w4.txt && exit 1
for lib in build/abw4/libw4.so citadels_self_play_amd/libcitadels_hip.so; do
  for c in 4 3; do
    CIT_LIB_PATH=$lib timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-pmc --cfr-reps 5 > $O/bench_$(basename $lib .so)_c$c.json 2> $O/bench_$(basename $lib .so)_c$c.err || exit 1
  done
done
