#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_targets.py tests/test_gpu_cfr.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "golden or fingerprint" > gpurun_out/gpu_tests_b.log 2>&1 &&
timeout -k 10 300 python -u tools/prof_cfr.py run > gpurun_out/cfr_phases2.jsonl 2> gpurun_out/cfr_phases2.err
