#!/bin/bash
# r3o: wide bf16 forward (copies) + backward: attention GPU tests, HSTU layer tests, C3 micro
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 500 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_hstu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3o_test.log 2>&1 || { grep -E "PASS|FAIL|Error|error|rel err" gpurun_out/r3o_test.log | tail -40; exit 1; }
grep -E "passed|failed" gpurun_out/r3o_test.log | tail -2
timeout -k 10 120 python -u scripts/attn_micro.py --shape c3 --bf16 --iters 10 > gpurun_out/r3o_micro.log 2>&1 || { tail -20 gpurun_out/r3o_micro.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3o_micro.log
