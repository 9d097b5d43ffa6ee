#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
TAG=r4f BENCH_ARGS="--no-retrieval-leg --e2e-steps 0 --c5-steps 0 --c3-steps 0 --no-bf16-leg --sweep 128 --no-cpu-baseline" \
  bash scripts/quick_bench.sh tests/test_gpu_topk.py tests/test_gpu_runner.py tests/test_gpu_postproc.py &&
TAG=r4e bash scripts/r4_attn_counters.sh
