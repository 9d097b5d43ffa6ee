#!/bin/bash
# SQ counters of the C3 attention backward (bf16 wide and f32 wide), run via gpurun.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r4e}
mkdir -p gpurun_out/$TAG
timeout -k 10 200 python3 scripts/attn_micro.py --shape c3 --bf16 --hepi --only bwd --iters 5 > gpurun_out/$TAG/micro_bf16.json &&
timeout -k 10 200 python3 scripts/attn_micro.py --shape c3 --hepi --only bwd --iters 3 > gpurun_out/$TAG/micro_f32.json &&
bash scripts/counters.sh $TAG/bf16 scripts/attn_micro.py --shape c3 --bf16 --hepi --only bwd --iters 2 &&
python3 scripts/counter_summary.py gpurun_out/$TAG/bf16/p1 gpurun_out/$TAG/bf16/p2 > gpurun_out/$TAG/bf16_summary.txt &&
bash scripts/counters.sh $TAG/f32 scripts/attn_micro.py --shape c3 --hepi --only bwd --iters 1 &&
python3 scripts/counter_summary.py gpurun_out/$TAG/f32/p1 gpurun_out/$TAG/f32/p2 > gpurun_out/$TAG/f32_summary.txt
