#!/bin/bash
# Rehearsal of bench.py's N = 2 path on the one-GPU box (GR_BENCH_SHARED_GPU: both ranks on
# cuda:0, gloo for the collectives); checks that every leg runs at world 2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6s
GR_BENCH_SHARED_GPU=1 timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline \
  --sweep= --c3-steps 2 --c5-steps 1 --e2e-steps 5 --retrieval-steps 3 > gpurun_out/r6s/bench2.log 2>&1 || { tail -30 gpurun_out/r6s/bench2.log; exit 1; }
grep '"metric"' gpurun_out/r6s/bench2.log | cut -c1-400
