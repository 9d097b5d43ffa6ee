#!/bin/bash
# r3y: round-3 profile of the headline (C2 step + C4 retrieval): kernel trace + FETCH / WRITE passes
set -o pipefail
cd "$(dirname "$0")/.."
bash scripts/profile_round.sh r3y "--steps 20 --warmup 5 --no-cpu-baseline --retrieval-steps 5 --c3-steps 0 --no-bf16-leg --e2e-steps 0 --c5-steps 0 --sweep= --retrieval-d256-items 0" || exit 1
grep '^{"metric' gpurun_out/r3y/bench_trace.log | cut -c1-300
