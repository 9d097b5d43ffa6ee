#!/bin/bash
# r3al: bf16 gate_o_bwd panel held to three waves per SIMD (18 spilled VGPRs): micro at C3, tests
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest tests/test_gpu_hstu.py -x -q -k "bf16" --timeout 200 --timeout-method thread > gpurun_out/r3al_test.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/r3al_test.log | tail -30; tail -3 gpurun_out/r3al_test.log; exit 1; }
tail -1 gpurun_out/r3al_test.log
for i in 1 2; do
timeout -k 10 120 python -u scripts/gemm_micro.py --shape c3 --iters 20 --bf16-panels > gpurun_out/r3al_micro.log 2>&1 || { tail -20 gpurun_out/r3al_micro.log; exit 1; }
tail -1 gpurun_out/r3al_micro.log
done
