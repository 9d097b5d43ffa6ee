#!/bin/bash
# pairs heuristic + options API: GPU suites touched, micro, timeline
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_hstu.py tests/test_gpu_topk.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2r_tests.log 2>&1
for B in 32 128; do
  timeout -k 5 90 python scripts/attn_micro.py --shape c2 --batch $B --only bwd --hepi --iters 20 >> gpurun_out/r2r_micro.jsonl
done
GR_HSTU_LIB=vlib/libgr_stamp.so timeout -k 5 90 python scripts/timeline_bwd.py --batch 128 >> gpurun_out/r2r_tl.jsonl
timeout -k 10 300 python bench.py --no-retrieval-leg --no-cpu-baseline --e2e-steps 0 --sweep "" --no-bf16-leg --c3-steps 0 > gpurun_out/r2r_bench.json 2> gpurun_out/r2r_bench.err
