#!/bin/bash
# r3t: dQ-in-key-major backward form (ATTN_BWD_DS=3): launch-mode test + C2 micro
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -x -v --timeout 200 --timeout-method thread -k "launch_modes or bwd" > gpurun_out/r3t_test.log 2>&1 || { grep -E "PASS|FAIL|Error|error|rel err|assert" gpurun_out/r3t_test.log | tail -30; exit 1; }
grep -E "passed|failed" gpurun_out/r3t_test.log | tail -2
run() { timeout -k 10 90 python -u scripts/attn_micro.py --shape c2 --only bwd --hepi --iters 30 "$@" 2>&1 | grep -v amdgpu.ids; }
{ echo base; run; echo ds3; run --ds 3; echo ds3pairs0; run --ds 3 --pairs 0; echo ds3pairs2; run --ds 3 --pairs 2; echo ds3b32; run --ds 3 --batch 32; echo ds3b512; run --ds 3 --batch 512; } > gpurun_out/r3t.log 2>&1 || { tail -20 gpurun_out/r3t.log; exit 1; }
cat gpurun_out/r3t.log
