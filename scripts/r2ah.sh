#!/bin/bash
# preact-only as an opt-in mode: parity (kernel + encoder level), default bench
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_preact.py tests/test_gpu_hstu.py tests/test_gpu_runner.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2ah_tests.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/r2ah_bench.json 2> gpurun_out/r2ah_bench.err
