#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4n
M=gpurun_out/r4n/micro.txt
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_attention.py tests/test_gpu_hstu.py tests/test_capi.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4n/test.log 2>&1 || { tail -30 gpurun_out/r4n/test.log; exit 1; }
tail -1 gpurun_out/r4n/test.log
timeout -k 10 120 python3 scripts/attn_micro.py --shape c2 --hepi --iters 50 --ds 1 >> $M || exit 1
timeout -k 10 120 python3 scripts/attn_micro.py --shape c2 --hepi --iters 50 --ds 1 --pairs 2 >> $M || exit 1
cat $M
GR_HSTU_LIB=stamplib/libgr_stamp.so timeout -k 10 120 python3 scripts/stamp_dkv.py --batch 128 --len 200 --hepi > gpurun_out/r4n/stamp.txt 2>&1 || { tail gpurun_out/r4n/stamp.txt; exit 1; }
cat gpurun_out/r4n/stamp.txt
TAG=r4n_b BENCH_ARGS="--e2e-steps 0 --c5-steps 0 --c3-steps 0" bash scripts/quick_bench.sh
