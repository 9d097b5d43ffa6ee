#!/bin/bash
# colsum from the A operand (no padding panel), preact-only opt-in: parity + bench
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_preact.py tests/test_gpu_hstu.py tests/test_gpu_attention.py tests/test_gpu_runner.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2ai_tests.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/r2ai_bench.json 2> gpurun_out/r2ai_bench.err
timeout -k 5 120 python scripts/attn_micro.py --shape c3 --bf16 --hepi --iters 5 > gpurun_out/r2ai_micro.jsonl
