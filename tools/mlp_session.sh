set -o pipefail
O=gpurun_out/${MLP_TAG:-mlp}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -x -v --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || exit 1
timeout -k 10 200 python tools/bench_mlp.py > $O/bench_mlp.jsonl 2> $O/bench_mlp.err || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_mlp.py > $GRAFT_REPO_ROOT/$O/prof_bench.jsonl 2> $GRAFT_REPO_ROOT/$O/prof.err
