#!/bin/bash
# Profiles bench.py on the GPU box (run via gpurun).  Three separate rocprofv3 passes:
#   1. kernel trace + stats  (per-kernel durations)
#   2. --pmc FETCH_SIZE      (HBM read bytes, its own pass)
#   3. --pmc WRITE_SIZE      (HBM write bytes, its own pass)
# Outputs under gpurun_out/$TAG/; copy the summaries into profiles/.
set -e
TAG=${1:-prof}
ARGS=${2:-"--steps 20 --warmup 5 --no-cpu-baseline --retrieval-steps 5"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/trace -o run \
  --output-format csv -- python3 bench.py $ARGS > gpurun_out/$TAG/bench_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/$TAG/fetch -o run \
  --output-format csv -- python3 bench.py $ARGS --eager > gpurun_out/$TAG/bench_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/$TAG/write -o run \
  --output-format csv -- python3 bench.py $ARGS --eager > gpurun_out/$TAG/bench_write.log 2>&1
echo profile done
