#!/bin/bash
# Configs 3-5 (median of reps after a warm-up), CFR kernel trace + counters.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/sp
mkdir -p $O
timeout -k 10 200 python tools/bench_selfplay.py --config 3 --reps 5 > $O/c3.json 2> $O/c3.err &&
timeout -k 10 300 python tools/bench_selfplay.py --config 4 --reps 3 > $O/c4.json 2> $O/c4.err &&
timeout -k 10 400 python tools/bench_selfplay.py --config 5 --reps 3 > $O/c5.json 2> $O/c5.err &&
cd /tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace3 -o run -- python3 $R/tools/bench_cfr.py --batch 1024 --reps 3 > $O/trace3.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace4 -o run -- python3 $R/tools/bench_cfr.py --pred --batch 4096 --node-cap 2048 --reps 2 > $O/trace4.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM --output-format csv -d $O/pmc_a -o run -- python3 $R/tools/bench_cfr.py --batch 1024 --reps 1 > $O/pmc_a.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH --output-format csv -d $O/pmc_b -o run -- python3 $R/tools/bench_cfr.py --batch 1024 --reps 1 > $O/pmc_b.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o run -- python3 $R/tools/bench_cfr.py --batch 1024 --reps 1 > $O/pmc_f.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o run -- python3 $R/tools/bench_cfr.py --batch 1024 --reps 1 > $O/pmc_w.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM --output-format csv -d $O/pmc4_a -o run -- python3 $R/tools/bench_cfr.py --pred --batch 4096 --node-cap 2048 --reps 1 > $O/pmc4_a.log 2>&1 &&
cd $R && for p in a b f w; do python3 tools/pmc_kernel_sum.py $O/pmc_$p k_cfr_decide > $O/sum_$p.json; done &&
python3 tools/pmc_kernel_sum.py $O/pmc4_a k_cfr_pred_step > $O/sum4_pred.json && python3 tools/pmc_kernel_sum.py $O/pmc4_a k_mlp > $O/sum4_mlp.json
