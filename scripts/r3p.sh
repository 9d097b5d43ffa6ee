#!/bin/bash
# r3p: wgrad XCD order: wgrad tests, then the C3 legs
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3p_test.log 2>&1 || { tail -30 gpurun_out/r3p_test.log; exit 1; }
tail -1 gpurun_out/r3p_test.log
bash scripts/r3m.sh
