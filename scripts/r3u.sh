#!/bin/bash
# r3u: f32 attention backward without the loop-entry waitcnt merge: tests + C2 micro
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3u_test.log 2>&1 || { grep -E "PASS|FAIL|Error|error|rel err|assert" gpurun_out/r3u_test.log | tail -30; exit 1; }
grep -E "passed|failed" gpurun_out/r3u_test.log | tail -2
run() { timeout -k 10 90 python -u scripts/attn_micro.py --shape c2 --hepi --iters 30 "$@" 2>&1 | grep -v amdgpu.ids; }
{ echo fused; run; echo split; run --split --only bwd; echo ds1; run --ds 1 --only bwd; echo b32; run --batch 32; echo b512; run --batch 512; } > gpurun_out/r3u.log 2>&1 || { tail -20 gpurun_out/r3u.log; exit 1; }
cat gpurun_out/r3u.log
