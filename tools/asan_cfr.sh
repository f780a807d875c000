#!/bin/bash
# The host build of the search under ASan + UBSan with given LDS buffer sizes
# (default: the round-3 4-waves experiment's CFR_LBUF=16 CFR_SBUF=32), configs
# 3 / 4 / 5 for SECONDS each (CPU only; writes build/asan_cfr_*.log).
#   tools/asan_cfr.sh [SECONDS] [LBUF] [SBUF]
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
S=${1:-20}
LB=${2:-16}
SB=${3:-32}
mkdir -p "$R/build"
g++ -O1 -g -std=c++17 -ffp-contract=off -fno-strict-aliasing -pthread -fsanitize=address,undefined \
  -fno-sanitize-recover=undefined -DCFR_LBUF="$LB" -DCFR_SBUF="$SB" "$R/tools/asan_cfr.cpp" -o "$R/build/asan_cfr"
"$R/build/asan_cfr" "$S" 2000 2>&1 | tee "$R/build/asan_cfr_l${LB}_s${SB}.log"
