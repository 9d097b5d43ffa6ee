#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4k
for pr in 1 0; do timeout -k 10 200 python3 scripts/topk_micro.py --dim 256 --iters 5 --opt MIPS_FILTER_PAIRED=$pr; done > gpurun_out/r4k/d256.txt; cat gpurun_out/r4k/d256.txt
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_attention.py tests/test_gpu_wgrad.py tests/test_gpu_wgrad_multi.py tests/test_gpu_hstu.py tests/test_gpu_topk.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4k/test.log 2>&1; tail -3 gpurun_out/r4k/test.log
TAG=r4k_b BENCH_ARGS="--e2e-steps 0 --c5-steps 0 --sweep 128 --no-cpu-baseline" bash scripts/quick_bench.sh
