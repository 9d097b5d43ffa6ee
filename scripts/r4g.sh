#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
TAG=r4g BENCH_ARGS="--no-retrieval-leg --e2e-steps 0 --c5-steps 0 --c3-steps 0 --no-bf16-leg --sweep 128 --no-cpu-baseline" \
  bash scripts/quick_bench.sh tests/test_gpu_topk.py tests/test_gpu_runner.py &&
bash scripts/profile_round.sh r4g_prof "--steps 20 --warmup 5 --no-cpu-baseline --retrieval-steps 5 --c3-steps 0 --e2e-steps 0 --c5-steps 0 --no-bf16-leg --sweep 128"
