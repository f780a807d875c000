#!/bin/bash
# instruction-cache evidence for k_rollout_u (one --pmc pass of 8 SQ-block counters)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/icache
mkdir -p $O
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $O/p1 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pmc > $O/p1.log 2>&1 &&
python3 $R/tools/pmc_kernel_sum.py $O/p1 k_rollout_u > $O/rollout.json &&
timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $O/p2 -o run -- python3 $R/tools/bench_cfr.py --batch 1024 --reps 1 > $O/p2.log 2>&1 &&
python3 $R/tools/pmc_kernel_sum.py $O/p2 k_cfr_decide > $O/cfr.json
