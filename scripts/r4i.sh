#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4i
timeout -k 10 120 python3 scripts/topk_micro.py --items 3953 --iters 20 > gpurun_out/r4i/small.txt &&
timeout -k 10 200 python3 scripts/topk_micro.py --iters 10 > gpurun_out/r4i/c4.txt &&
bash scripts/counters.sh r4i/small scripts/topk_micro.py --items 3953 --iters 3 &&
python3 scripts/counter_summary.py gpurun_out/r4i/small/p1 gpurun_out/r4i/small/p2 > gpurun_out/r4i/small_summary.txt &&
bash scripts/counters.sh r4i/c4 scripts/topk_micro.py --iters 2 &&
python3 scripts/counter_summary.py gpurun_out/r4i/c4/p1 gpurun_out/r4i/c4/p2 > gpurun_out/r4i/c4_summary.txt
