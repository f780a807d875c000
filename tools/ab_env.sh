#!/bin/bash
# Interleaved A/B of an environment setting over bench.py runs on the GPU box:
#   tools/ab_env.sh TAG VAR "V1 V2 ..." REPS BENCH_ARGS...
# -> gpurun_out/TAG/VAR=V_rep.json (one bench line each) and summary.txt
# (value per run).  Each run has its own time limit; the first failure ends it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1 VAR=$2 VALS=$3 REPS=$4
shift 4
O=$R/gpurun_out/$TAG
mkdir -p "$O"
for rep in $(seq 1 "$REPS"); do
  for v in $VALS; do
    (cd "$R" && env "$VAR=$v" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pmc "$@" \
      > "$O/${VAR}=${v}_$rep.json" 2> "$O/${VAR}=${v}_$rep.err") || exit 1
  done
done
for v in $VALS; do
  echo "$VAR=$v $(for rep in $(seq 1 "$REPS"); do tail -1 "$O/${VAR}=${v}_$rep.json" | python3 -c \
    'import json,sys; print(round(json.loads(sys.stdin.read())["value"], 1))'; done | tr '\n' ' ')"
done > "$O/summary.txt"
