#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4w
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_hstu.py tests/test_gpu_topk.py tests/test_capi.py tests/test_gpu_distributed.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4w/test.log 2>&1 || { tail -30 gpurun_out/r4w/test.log; exit 1; }
tail -1 gpurun_out/r4w/test.log
timeout -k 10 200 python3 scripts/topk_micro.py --iters 20 > gpurun_out/r4w/micro.txt || exit 1
cat gpurun_out/r4w/micro.txt
bash scripts/round_bench.sh r4w_b
