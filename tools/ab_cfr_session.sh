# A/B of search builds (tools/ab_build.py with AB_UNIT=cit_cfr.hip): the CFR
# parity tests on the variant, then config 3 (and the config-5 trace) for
# base and variant, interleaved.  ab_cfr_session.sh VARIANT.so
O=gpurun_out/${AB_TAG:-abcfr}; mkdir -p $O
V=$1
CIT_LIB_PATH=$V timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "cfr or targets or config" --timeout 300 --timeout-method thread > $O/tests_variant.txt 2>&1 || exit 1
for rep in 1 2; do
  for lib in citadels_self_play_amd/libcitadels_hip.so $V; do
    n=$(basename $lib .so)_$rep
    CIT_LIB_PATH=$lib timeout -k 10 300 python bench.py --config 3 --no-pmc --no-cpu-baseline --cfr-reps 5 > $O/c3_$n.json 2> $O/c3_$n.err || exit 1
  done
done
