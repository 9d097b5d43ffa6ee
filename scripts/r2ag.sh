#!/bin/bash
# pre-activation hand-over (ABI 9): parity + attention micro A/B + default bench
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_preact.py tests/test_gpu_attention.py tests/test_gpu_hstu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2ag_tests.log 2>&1
for A in "" "--act"; do
  timeout -k 5 90 python scripts/attn_micro.py --shape c2 --hepi --iters 20 $A >> gpurun_out/r2ag_micro.jsonl
  timeout -k 5 90 python scripts/attn_micro.py --shape c3 --hepi --iters 5 $A >> gpurun_out/r2ag_micro.jsonl
done
timeout -k 10 600 python bench.py > gpurun_out/r2ag_bench.json 2> gpurun_out/r2ag_bench.err
