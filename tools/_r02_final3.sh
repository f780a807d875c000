#!/bin/bash
# Round-2 closing evidence: GPU suite, smoke, default bench (3 streams, in-run
# PMC, CPU baseline), rocprofv3 kernel traces of the bench (one stream and default).
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/final3
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err &&
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_s1 -o run -- python3 $R/bench.py --streams 1 --no-cpu-baseline --no-pmc > $O/trace_s1.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_s2 -o run -- python3 $R/bench.py --no-cpu-baseline --no-pmc > $O/trace_s2.log 2>&1
