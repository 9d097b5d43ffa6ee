#!/bin/bash
# one-launch dS hand-off backward: parity (all launch forms) + micro A/B + bench
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 120 --timeout-method thread -k "launch_modes or bwd" > gpurun_out/r2aa_tests.log 2>&1
for args in "" "--ds 1" "--ds 2" "--ds 2 --pairs 2"; do
  timeout -k 5 90 python scripts/attn_micro.py --shape c2 --batch 128 --only bwd --hepi --iters 20 $args >> gpurun_out/r2aa_micro.jsonl
done
