#!/bin/bash
# GPU check after a search change: full GPU suite, per-tree clock, phase profile, bench.
set -o pipefail
O=gpurun_out/chk
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 200 python -u tools/cfr_tree_clock.py run > $O/treeclock.jsonl 2> $O/treeclock.err &&
timeout -k 10 300 python -u tools/prof_cfr.py run > $O/prof.jsonl 2> $O/prof.err &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc > $O/bench.log 2>&1
