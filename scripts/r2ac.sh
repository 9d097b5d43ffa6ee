#!/bin/bash
# small-catalog retrieval: chunked score-all (parity + timing)
set -e
cd $GRAFT_REPO_ROOT
true
timeout -k 5 120 python scripts/topk_micro.py --items 3953 --iters 50 > gpurun_out/r2ac_micro.txt 2>&1
timeout -k 5 120 python scripts/topk_micro.py --items 27278 --n0 2059 --iters 20 >> gpurun_out/r2ac_micro.txt 2>&1
