#!/bin/bash
# C2 headline leg only, once per launch-option setting (A/B on the GPU box):
#   gpurun -- 'TAG=r5b bash scripts/c2_sweep.sh "" "WGRAD_ROWS=800" "WGRAD_ROWS=1600"'
# Each argument is a space-separated list of NAME=VALUE options ("" = defaults).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-sweep}
mkdir -p gpurun_out/$TAG
i=0
for opts in "$@"; do
  args=""
  for o in $opts; do args="$args --opt $o"; done
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-retrieval-leg --no-bf16-leg \
    --c3-steps 0 --c5-steps 0 --e2e-steps 0 --sweep "" --retrieval-d256-items 0 \
    --steps ${STEPS:-50} ${BENCH_ARGS:-} $args > gpurun_out/$TAG/run$i.log 2>&1 \
    || { tail -20 gpurun_out/$TAG/run$i.log; exit 1; }
  tail -1 gpurun_out/$TAG/run$i.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
k=d['roofline']['per_step_device_ms']
print('[$opts]', d['value'], d['ms_per_step'], {n: k[n] for n in list(k)[:12]})"
  i=$((i+1))
done
