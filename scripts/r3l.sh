#!/bin/bash
# r3l: wide bf16 backward: parity (bf16 attention tests) + C3 micro, bias and no-bias
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u -m pytest tests/test_gpu_attention.py -x -v -k "bf16" --timeout 200 --timeout-method thread > gpurun_out/r3l_test.log 2>&1 || { grep -E "PASS|FAIL|Error|error|rel err" gpurun_out/r3l_test.log | tail -40; exit 1; }
grep -E "passed|failed" gpurun_out/r3l_test.log | tail -2
run() { timeout -k 10 120 python -u scripts/attn_micro.py --shape c3 --bf16 --only bwd --iters 10 "$@"; }
{ run; run --nobias; } > gpurun_out/r3l_micro.log 2>&1 || { tail -20 gpurun_out/r3l_micro.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3l_micro.log
