#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4v
M=gpurun_out/r4v/micro.txt
for w in 2 3 4; do echo "WGS $w" >> $M; timeout -k 10 200 python3 scripts/topk_micro.py --iters 20 --opt MIPS_FILTER_WGS=$w >> $M || exit 1; done
cat $M
