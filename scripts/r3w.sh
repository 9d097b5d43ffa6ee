#!/bin/bash
# r3w: batched silu'(h) epilogues of the bf16 attention backward: tests + C3/C2 bf16 micro
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3w_test.log 2>&1 || { grep -E "PASS|FAIL|Error|error|rel err|assert" gpurun_out/r3w_test.log | tail -30; exit 1; }
grep -E "passed|failed" gpurun_out/r3w_test.log | tail -2
run() { timeout -k 10 90 python -u scripts/attn_micro.py --hepi "$@" 2>&1 | grep -v amdgpu.ids; }
{ echo c3bf16; run --shape c3 --bf16 --iters 10; echo c2bf16; run --shape c2 --bf16 --iters 30; } > gpurun_out/r3w.log 2>&1 || { tail -20 gpurun_out/r3w.log; exit 1; }
cat gpurun_out/r3w.log
