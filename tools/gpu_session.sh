#!/bin/bash
# One parametrised runner for the GPU box (replaces round 1-2's one-off
# _r02_* / _run_* scripts).  Every GPU step runs under its own time limit and
# the steps are chained with &&: the first failure, timeout or fault ends the
# session.  Output goes to gpurun_out/$TAG/.
#
#   tools/gpu_session.sh TAG STEP [STEP ...]
#
# Steps:
#   tests[=EXPR]     pytest -m gpu (optionally -k EXPR)          -> tests.txt
#   smoke            __graft_entry__.smoke()                     -> smoke.log
#   bench[=ARGS]     python bench.py ARGS (commas become spaces) -> bench.json
#   trace[=ARGS]     rocprofv3 --kernel-trace --stats over bench.py ARGS -> trace/
#   pmc=CTRS[:ARGS]  one rocprofv3 --pmc pass (CTRS comma-separated, one block's
#                    worth) over bench.py ARGS                    -> pmc_<n>/
#   dist             N=2 gloo rehearsal of the multi-rank paths (ranks folded
#                    onto cuda:0; the real N>1 path is RCCL, one rank per GPU)
#   ab=LIBS          tools/_ablib.py A/B of rollout builds (colon-separated .so
#                    paths), 3 interleaved reps each           -> ab/summary.txt
#   py=SCRIPT[:ARGS] python SCRIPT ARGS                          -> py_<n>.log
#   pyprof=SCRIPT[:ARGS] the same under rocprofv3 --kernel-trace --stats -> pyprof_<n>/
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
n=0
run_step() {
  local step=$1 key=${1%%=*} val=
  [[ $step == *=* ]] && val=${step#*=}
  n=$((n + 1))
  echo "[$(date +%T)] step $n: $step" >> "$O/session.log"
  case $key in
    tests)
      if [ -n "$val" ]; then
        (cd "$R" && timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v -s -k "$val" --timeout 900 \
          --timeout-method thread > "$O/tests.txt" 2>&1)
      else
        (cd "$R" && timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v -s --timeout 900 \
          --timeout-method thread > "$O/tests.txt" 2>&1)
      fi ;;
    smoke)
      (cd "$R" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1) ;;
    bench)
      (cd "$R" && timeout -k 10 900 python -u bench.py --full-out "$O/bench_full.json" ${val//,/ } > "$O/bench.json" \
        2> "$O/bench.err") \
        && { for f in /tmp/bench_trace_*/*/*kernel_stats.csv /tmp/bench_trace_*/*kernel_stats.csv; do
               [ -f "$f" ] && cp "$f" "$O/bench_rollout_kernel_stats.csv"; done; true; } ;;
    trace)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
        python3 "$R/bench.py" --no-cpu-baseline --no-pmc ${val//,/ } > "$O/trace.log" 2>&1) ;;
    pmc)
      local ctrs=${val%%:*} args=
      [[ $val == *:* ]] && args=${val#*:}
      (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc ${ctrs//,/ } --output-format csv -d "$O/pmc_$n" -o run -- \
        python3 "$R/bench.py" --no-cpu-baseline --no-pmc --no-cfr ${args//,/ } > "$O/pmc_$n.log" 2>&1) ;;
    dist)
      (cd "$R" && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo \
        --cfg5-trees 32 --cfg5-iters 2000 --cfr-reps 1 > "$O/dist_bench.json" 2> "$O/dist_bench.err") ;;
    ab)
      mkdir -p "$O/ab"
      local libs=${val//:/ } ok=0
      for rep in 1 2 3; do
        for v in $libs; do
          (cd "$R" && timeout -k 10 120 python tools/_ablib.py "$v" 4096 > "$O/ab/$(basename "$v" .so)_$rep.log" 2>&1) \
            || { ok=1; break 2; }
        done
      done
      [ $ok -eq 0 ] && for v in $libs; do
        echo "$(basename "$v" .so) $(for rep in 1 2 3; do tail -1 "$O/ab/$(basename "$v" .so)_$rep.log" | python3 -c \
          'import json,sys; print(round(json.loads(sys.stdin.read())["value"]/1e6,1))'; done | tr '\n' ' ')"
      done > "$O/ab/summary.txt"
      return $ok ;;
    py)
      local script=${val%%:*} args=
      [[ $val == *:* ]] && args=${val#*:}
      (cd "$R" && timeout -k 10 900 python -u "$script" ${args//,/ } > "$O/py_$n.log" 2>&1) ;;
    pyprof)
      local script=${val%%:*} args=
      [[ $val == *:* ]] && args=${val#*:}
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/pyprof_$n" -o run -- \
        python3 "$R/$script" ${args//,/ } > "$O/pyprof_$n.log" 2>&1) ;;
    *)
      echo "unknown step $step" >&2
      return 2 ;;
  esac
}
for s in "$@"; do
  run_step "$s" || { echo "[$(date +%T)] step $s FAILED (exit $?)" >> "$O/session.log"; exit 1; }
done
echo "[$(date +%T)] all steps done" >> "$O/session.log"
