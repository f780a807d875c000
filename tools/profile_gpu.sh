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
GPB=${GPB:-16}
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
