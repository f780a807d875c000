#!/bin/bash
# CFR counter evidence on the box: per-tree clock distribution, kernel trace,
# SQ / icache / HBM counters of k_cfr_decide (config 3, 1024 trees).
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/cfrpmc
mkdir -p $O
timeout -k 10 200 python -u tools/cfr_tree_clock.py run > $O/treeclock.jsonl 2> $O/treeclock.err &&
cd /tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace3 -o run -- python3 $R/tools/bench_cfr.py --batch 1024 --reps 3 > $O/trace3.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM --output-format csv -d $O/pmc_a -o run -- python3 $R/tools/bench_cfr.py --batch 1024 --reps 1 > $O/pmc_a.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH --output-format csv -d $O/pmc_b -o run -- python3 $R/tools/bench_cfr.py --batch 1024 --reps 1 > $O/pmc_b.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $O/pmc_c -o run -- python3 $R/tools/bench_cfr.py --batch 1024 --reps 1 > $O/pmc_c.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o run -- python3 $R/tools/bench_cfr.py --batch 1024 --reps 1 > $O/pmc_f.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o run -- python3 $R/tools/bench_cfr.py --batch 1024 --reps 1 > $O/pmc_w.log 2>&1 &&
cd $R && for p in a b c f w; do python3 tools/pmc_kernel_sum.py $O/pmc_$p k_cfr_decide > $O/sum_$p.json; done
