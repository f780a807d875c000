#!/bin/bash
# rocprofv3 passes for the rollout kernel, run on the GPU box:
#   1. --kernel-trace --stats (per-kernel durations)
#   2. --pmc FETCH_SIZE   (own pass: TCC slots)
#   3. --pmc WRITE_SIZE   (own pass)
# then tools/pmc_summary.py folds them into gpurun_out/prof/summary.json.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof
STEPS=${STEPS:-5}
GPB=${GPB:-0}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$R/bench.py" --steps "$STEPS" --warmup 1 --no-cpu-baseline --games-per-block "$GPB" > "$OUT/trace_bench.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --games-per-block "$GPB" > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --games-per-block "$GPB" > "$OUT/pmc_write.log" 2>&1
python3 "$R/tools/pmc_summary.py" "$OUT" > "$OUT/summary.json"
cat "$OUT/summary.json"
# MCCFR kernels (config 3 no-model, config 4 with value-net leaves): durations only
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_cfr" -o run -- \
  python3 "$R/tools/bench_cfr.py" --batch 1024 --reps 2 > "$OUT/trace_cfr3.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_pred" -o run -- \
  python3 "$R/tools/bench_cfr.py" --pred --batch 4096 --node-cap 2048 --reps 2 > "$OUT/trace_cfr4.log" 2>&1
