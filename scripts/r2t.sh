#!/bin/bash
# bf16 projections: encoder parity (bf16 mode) + C3/C2 bf16 legs
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_hstu.py tests/test_gpu_attention.py -x -q -s -k "bf16" --timeout 300 --timeout-method thread > gpurun_out/r2t_tests.log 2>&1
timeout -k 10 400 python bench.py --no-retrieval-leg --no-cpu-baseline --e2e-steps 0 --sweep "" --steps 20 > gpurun_out/r2t_bench.json 2> gpurun_out/r2t_bench.err
