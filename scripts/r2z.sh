#!/bin/bash
# rehearsal of bench.py's N = 2 path on one GPU (gloo, both ranks on cuda:0)
set -e
cd $GRAFT_REPO_ROOT
export GR_BENCH_SHARED_GPU=1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --retrieval-steps 2 --c3-steps 2 --e2e-steps 2 --sweep , > gpurun_out/r2z_bench2.json 2> gpurun_out/r2z_bench2.err
