#!/bin/bash
# The C2 headline leg alone (other legs off), interleaved over bench argument sets:
#   gpurun -- 'bash scripts/c2_only.sh "" "--opt ATTN_BWD_PAIRS=2"'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/c2only
for rep in 1 2; do
  for a in "$@"; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-retrieval-leg --e2e-steps 0 --sweep "" \
      --c3-steps 0 --no-bf16-leg --c5-steps 0 $a > gpurun_out/c2only/run.log 2>&1 \
      || { tail -20 gpurun_out/c2only/run.log; exit 1; }
    tail -1 gpurun_out/c2only/run.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('[$a]', d['value'], d['ms_per_step'])"
  done
done
