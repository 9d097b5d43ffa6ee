#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4m
M=gpurun_out/r4m/micro.txt
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_topk.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4m/test_topk.log 2>&1 || { tail -30 gpurun_out/r4m/test_topk.log; exit 1; }
tail -1 gpurun_out/r4m/test_topk.log
timeout -k 10 200 python3 scripts/topk_micro.py --iters 20 >> $M || exit 1
timeout -k 10 200 python3 scripts/topk_micro.py --dim 256 --iters 5 >> $M || exit 1
for sp in 0 1 2; do timeout -k 10 120 python3 scripts/attn_micro.py --shape c3 --hepi --only bwd --iters 3 --opt ATTN_BWD_WIDE_SPLIT=$sp >> $M || exit 1; done
timeout -k 10 120 python3 scripts/attn_micro.py --shape c2 --hepi --iters 50 >> $M || exit 1
timeout -k 10 120 python3 scripts/attn_micro.py --shape c2 --hepi --iters 50 --bf16 >> $M || exit 1
timeout -k 10 120 python3 scripts/attn_micro.py --shape c2 --hepi --iters 50 --ds 1 >> $M || exit 1
timeout -k 10 120 python3 scripts/attn_micro.py --shape c2 --hepi --iters 50 --ds 2 >> $M || exit 1
cat $M
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_attention.py -m gpu -x -q --timeout 200 --timeout-method thread -k "wide" > gpurun_out/r4m/test_attn.log 2>&1 || { tail -30 gpurun_out/r4m/test_attn.log; exit 1; }
tail -1 gpurun_out/r4m/test_attn.log
TAG=r4m_b BENCH_ARGS="--e2e-steps 0 --c5-steps 0" bash scripts/quick_bench.sh
