#!/bin/bash
# Round-2 evidence on the box: GPU suite, smoke, bench (in-run PMC + CPU
# baseline), rollout kernel trace, configs 3-5, CFR / MLP kernel traces.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/final
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 &&
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace2 -o run -- python3 $R/bench.py --no-cpu-baseline --no-pmc > $O/trace2.log 2>&1 && cd $R &&
timeout -k 10 200 python tools/bench_selfplay.py --config 3 --reps 5 > $O/c3.json 2> $O/c3.err &&
timeout -k 10 300 python tools/bench_selfplay.py --config 4 --reps 3 > $O/c4.json 2> $O/c4.err &&
timeout -k 10 400 python tools/bench_selfplay.py --config 5 --reps 3 > $O/c5.json 2> $O/c5.err &&
timeout -k 10 400 python tools/bench_selfplay.py --config 5 --iters 200000 --reps 1 --warmup 0 > $O/c5_200k.json 2> $O/c5_200k.err &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace4 -o run -- python3 $R/tools/bench_cfr.py --pred --batch 4096 --node-cap 2048 --reps 2 > $O/trace4.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace3 -o run -- python3 $R/tools/bench_cfr.py --batch 1024 --reps 3 > $O/trace3.log 2>&1
