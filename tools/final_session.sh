# Round-end check on the final tree: full GPU suite, smoke, default bench,
# and the rocprofv3 kernel-trace summary of the rollout bench (its
# k_rollout_u average must agree with the bench line's kernel_avg_ms).
set -o pipefail
T=${FINAL_TAG:-final}
bash tools/gpu_session.sh $T tests smoke bench || exit 1
O=gpurun_out/$T; mkdir -p $O/prof
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cfr --no-pmc --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_bench.json 2> $GRAFT_REPO_ROOT/$O/prof_bench.err
