#!/bin/bash
# two-pass (dS) f32 attention backward: parity + micro A/B + encoder bench
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_hstu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2w_tests.log 2>&1
for B in 32 128 512; do
  timeout -k 5 90 python scripts/attn_micro.py --shape c2 --batch $B --only bwd --hepi --iters 20 --ds >> gpurun_out/r2w_micro.jsonl
done
timeout -k 5 90 python scripts/attn_micro.py --shape c2 --batch 128 --only bwd --hepi --iters 20 --ds --pairs 2 >> gpurun_out/r2w_micro.jsonl
timeout -k 5 90 python scripts/attn_micro.py --shape c2 --batch 128 --only bwd --hepi --iters 20 >> gpurun_out/r2w_micro.jsonl
timeout -k 10 300 python bench.py --no-retrieval-leg --no-cpu-baseline --e2e-steps 0 --sweep , --c3-steps 0 --no-bf16-leg > gpurun_out/r2w_bench.json 2> gpurun_out/r2w_bench.err
