set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_FLAT SQ_INSTS_FLAT_NO_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT SQ_ACTIVE_INST_LDS --output-format csv -d $R/gpurun_out/pmc_sq2 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_sq2.log 2>&1
