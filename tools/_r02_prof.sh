#!/bin/bash
# CFR evidence: phase cycles (CIT_PROF build), rocprofv3 kernel stats + PMC of
# k_cfr_decide (config 3) and k_cfr_pred_step / k_mlp (config 4); then the
# config-5 200k error diagnosis.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/cfr
mkdir -p $O
timeout -k 10 300 python -u tools/prof_cfr.py run > $O/phases.jsonl 2> $O/phases.err &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace3 -o run -- python3 $R/tools/bench_cfr.py --batch 1024 --reps 2 > $O/trace3.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace4 -o run -- python3 $R/tools/bench_cfr.py --pred --batch 4096 --node-cap 2048 --reps 2 > $O/trace4.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM --output-format csv -d $O/pmc_sq3 -o run -- python3 $R/tools/bench_cfr.py --batch 1024 --reps 1 > $O/pmc_sq3.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH --output-format csv -d $O/pmc_sq3b -o run -- python3 $R/tools/bench_cfr.py --batch 1024 --reps 1 > $O/pmc_sq3b.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch3 -o run -- python3 $R/tools/bench_cfr.py --batch 1024 --reps 1 > $O/pmc_fetch3.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write3 -o run -- python3 $R/tools/bench_cfr.py --batch 1024 --reps 1 > $O/pmc_write3.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch4 -o run -- python3 $R/tools/bench_cfr.py --pred --batch 4096 --node-cap 2048 --reps 1 > $O/pmc_fetch4.log 2>&1 &&
cd $R &&
timeout -k 10 400 python -u tools/diag_cfr_errors.py 200000 64 > $O/diag200k.json 2> $O/diag200k.err
