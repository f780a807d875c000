set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pcs
timeout -k 10 60 rocprofv3 -L > gpurun_out/pcs/list.txt 2>&1
cd /tmp && timeout -s KILL 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 10 --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pcs/out -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/pcs/run.log 2>&1
echo rc=$? >> $GRAFT_REPO_ROOT/gpurun_out/pcs/run.log
ls -laR $GRAFT_REPO_ROOT/gpurun_out/pcs > $GRAFT_REPO_ROOT/gpurun_out/pcs/ls.txt
