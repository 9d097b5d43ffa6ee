#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4o
M=gpurun_out/r4o/micro.txt
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_attention.py tests/test_gpu_hstu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4o/test.log 2>&1 || { tail -30 gpurun_out/r4o/test.log; exit 1; }
tail -1 gpurun_out/r4o/test.log
timeout -k 10 120 python3 scripts/attn_micro.py --shape c2 --hepi --iters 50 >> $M || exit 1
timeout -k 10 120 python3 scripts/attn_micro.py --shape c3 --hepi --iters 3 >> $M || exit 1
cat $M
GR_HSTU_LIB=stamplib/libgr_stamp.so timeout -k 10 120 python3 scripts/stamp_dkv.py --batch 128 --len 200 --hepi > gpurun_out/r4o/stamp.txt 2>&1 || { tail gpurun_out/r4o/stamp.txt; exit 1; }
cat gpurun_out/r4o/stamp.txt
Q="--no-cpu-baseline --no-retrieval-leg --no-bf16-leg --e2e-steps 0 --c5-steps 0 --c3-steps 0 --sweep= --retrieval-d256-items 0"
for o in ATTN_BWD_DS=0 ATTN_BWD_DS=1; do
  timeout -k 10 300 python3 -u bench.py $Q --opt $o > gpurun_out/r4o/bench_$o.log 2>&1 || { tail -20 gpurun_out/r4o/bench_$o.log; exit 1; }
  tail -1 gpurun_out/r4o/bench_$o.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$o', d['value'], d['ms_per_step'], d['roofline']['per_step_device_ms_total'])"
done
