#!/bin/bash
# Two rocprofv3 --pmc passes of SQ counters over the config-2 bench (8 SQ counters
# per pass, each pass its own run); summary -> gpurun_out/sq/summary.json
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/sq
mkdir -p $OUT
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d $OUT/a -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/a.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES --output-format csv -d $OUT/b -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/b.log 2>&1 &&
python3 - "$OUT" <<'PY' > $OUT/summary.json
import csv, glob, json, os, sys, collections
d = sys.argv[1]
acc = collections.defaultdict(list)
for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(p)):
        if "k_rollout_u" in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(json.dumps({k: sum(v) / len(v) for k, v in sorted(acc.items())}, indent=1))
PY
