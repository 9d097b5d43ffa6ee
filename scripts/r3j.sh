#!/bin/bash
# r3j: wide-head bf16 attention backward (32x32x16 path): parity + C3 micro timing
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u -m pytest tests/test_gpu_attention.py -x -v -k "bf16" --timeout 200 --timeout-method thread > gpurun_out/r3j_test.log 2>&1 || { grep -E "PASS|FAIL|Error|error|rel err" gpurun_out/r3j_test.log | tail -40; exit 1; }
grep -E "passed|failed" gpurun_out/r3j_test.log | tail -2
timeout -k 10 200 python -u scripts/attn_micro.py --shape c3 --bf16 --iters 10 > gpurun_out/r3j_micro.log 2>&1 || { tail -20 gpurun_out/r3j_micro.log; exit 1; }
cat gpurun_out/r3j_micro.log
