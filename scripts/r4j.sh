#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4j
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_attention.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4j/test.log 2>&1 || { tail -30 gpurun_out/r4j/test.log; exit 1; }
tail -1 gpurun_out/r4j/test.log
timeout -k 10 120 python3 scripts/attn_micro.py --shape c2 --hepi --iters 20 > gpurun_out/r4j/micro_c2.txt; cat gpurun_out/r4j/micro_c2.txt
for sp in 1 2 0; do timeout -k 10 120 python3 scripts/attn_micro.py --shape c3 --hepi --only bwd --iters 3 --opt ATTN_BWD_WIDE_SPLIT=$sp; done > gpurun_out/r4j/micro.txt
cat gpurun_out/r4j/micro.txt
timeout -k 10 200 python3 scripts/topk_micro.py --items 3953 --iters 20 > gpurun_out/r4j/small.txt && cat gpurun_out/r4j/small.txt
timeout -k 10 200 python3 scripts/topk_micro.py --iters 10 > gpurun_out/r4j/c4.txt && cat gpurun_out/r4j/c4.txt
for pr in 1 0; do timeout -k 10 200 python3 -c "
import sys; sys.argv=['x','--dim','256','--iters','5']
from mygenerativerecommenders_amd import _lib; _lib.set_option('MIPS_FILTER_PAIRED', $pr)
exec(open('scripts/topk_micro.py').read())"; done > gpurun_out/r4j/d256.txt && cat gpurun_out/r4j/d256.txt
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_topk.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4j/test_topk.log 2>&1; tail -3 gpurun_out/r4j/test_topk.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_attention.py tests/test_gpu_rel_bias.py -m gpu -x -q --timeout 200 --timeout-method thread -k "bucket or rel_bias" > gpurun_out/r4j/test_bucket.log 2>&1; tail -3 gpurun_out/r4j/test_bucket.log
TAG=r4j_b BENCH_ARGS="--no-retrieval-leg --e2e-steps 0 --c5-steps 0 --c3-steps 0 --no-bf16-leg --sweep 128 --no-cpu-baseline" bash scripts/quick_bench.sh
for r in 128 192 256; do TAG=r4j_w$r BENCH_ARGS="--no-retrieval-leg --e2e-steps 0 --c5-steps 0 --c3-steps 0 --no-bf16-leg --sweep 128 --no-cpu-baseline --opt WGRAD_ROWS=$r" bash scripts/quick_bench.sh | head -2; done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_loss.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4j/test_loss.log 2>&1; tail -3 gpurun_out/r4j/test_loss.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_wgrad_multi.py tests/test_gpu_hstu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4j/test_wgrad.log 2>&1; tail -3 gpurun_out/r4j/test_wgrad.log
