#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4l
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_attention.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4l/test_attn.log 2>&1 || { tail -30 gpurun_out/r4l/test_attn.log; exit 1; }
tail -1 gpurun_out/r4l/test_attn.log
for sp in 2 3; do timeout -k 10 120 python3 scripts/attn_micro.py --shape c3 --hepi --only bwd --iters 3 --opt ATTN_BWD_WIDE_SPLIT=$sp; done | tee gpurun_out/r4l/micro.txt
for pr in 1 0; do timeout -k 10 200 python3 scripts/topk_micro.py --dim 256 --iters 5 --opt MIPS_FILTER_PAIRED=$pr; done | tee gpurun_out/r4l/d256.txt
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_wgrad_multi.py tests/test_gpu_hstu.py tests/test_gpu_topk.py tests/test_gpu_distributed.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4l/test.log 2>&1; tail -3 gpurun_out/r4l/test.log
TAG=r4l_b BENCH_ARGS="--e2e-steps 0 --c5-steps 0 --sweep 128 --no-cpu-baseline" bash scripts/quick_bench.sh
