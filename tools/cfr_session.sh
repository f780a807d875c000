# Search-side check after a change: CFR/targets/config parity tests, the
# config-5 trace, and bench.py's CFR legs (config 3 as the headline line).
O=gpurun_out/${CFR_TAG:-cfr}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "cfr or targets or config or api or selfplay or train or queue" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || exit 1
timeout -k 10 200 python tools/cfg5_trace.py 1920 200000 $O/cfg5 > $O/cfg5.json 2> $O/cfg5.err || exit 1
timeout -k 10 400 python bench.py --config 3 --no-pmc --no-cpu-baseline --cfr-configs 3,4,5 > $O/bench.json 2> $O/bench.err || exit 1
