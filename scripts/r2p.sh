#!/bin/bash
# f32 attention backward, tile pairs: parity, micro A/B, timeline
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2q_tests.log 2>&1
for B in 32 128 512; do
  timeout -k 5 90 python scripts/attn_micro.py --shape c2 --batch $B --only bwd --hepi --iters 20 >> gpurun_out/r2q_micro.jsonl
done
timeout -k 5 90 python scripts/attn_micro.py --shape c2 --batch 128 --only bwd --hepi --iters 20 --nopairs >> gpurun_out/r2q_micro.jsonl
timeout -k 5 90 python scripts/attn_micro.py --shape c3 --only bwd --hepi --iters 5 >> gpurun_out/r2q_micro.jsonl
timeout -k 5 90 python scripts/attn_micro.py --shape c3 --only bwd --hepi --iters 5 --nopairs >> gpurun_out/r2q_micro.jsonl
GR_HSTU_LIB=vlib/libgr_stamp.so timeout -k 5 90 python scripts/timeline_bwd.py --batch 128 >> gpurun_out/r2q_tl.jsonl
