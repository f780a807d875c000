#!/bin/bash
set -o pipefail
O=gpurun_out/prof200k
mkdir -p $O
timeout -k 10 250 python -u tools/prof_cfr.py run top 200000:64 > $O/top.jsonl 2> $O/top.err &&
timeout -k 10 250 python -u tools/prof_cfr.py run node 200000:64 > $O/node.jsonl 2> $O/node.err
