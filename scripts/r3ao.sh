#!/bin/bash
# r3ao: C3 (fp32 + bf16) profile at the round-3 HEAD: kernel trace + FETCH / WRITE passes
set -o pipefail
cd "$(dirname "$0")/.."
bash scripts/profile_round.sh r3ao_c3 "--steps 2 --warmup 1 --no-cpu-baseline --no-retrieval-leg --c3-steps 3 --e2e-steps 0 --c5-steps 0 --sweep=" || exit 1
grep '^{"metric' gpurun_out/r3ao_c3/bench_trace.log | cut -c1-200
