#!/bin/bash
# r3v: f32 attention tests + C2 micro (loop-entry waitcnt fix), C3 bf16 micro with and
# without VGPR-form MFMAs in the wide bf16 kernels
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3v_test.log 2>&1 || { grep -E "PASS|FAIL|Error|error|rel err|assert" gpurun_out/r3v_test.log | tail -30; exit 1; }
grep -E "passed|failed" gpurun_out/r3v_test.log | tail -2
run() { timeout -k 10 90 python -u scripts/attn_micro.py --hepi "$@" 2>&1 | grep -v amdgpu.ids; }
{ echo c2; run --shape c2 --iters 30; echo c2split; run --shape c2 --iters 30 --split --only bwd; echo c2b32; run --shape c2 --iters 30 --batch 32;
  echo c3bf16; run --shape c3 --bf16 --iters 10; echo c3bf16_noform; GR_HSTU_LIB=vlib/libgr_noform.so run --shape c3 --bf16 --iters 10; } > gpurun_out/r3v.log 2>&1 || { tail -20 gpurun_out/r3v.log; exit 1; }
cat gpurun_out/r3v.log
