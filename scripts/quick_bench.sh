#!/bin/bash
# Tests (optional selectors) then a bench run without the CPU baseline, on the GPU box.
#   gpurun -- 'TAG=r4c bash scripts/quick_bench.sh tests/test_gpu_hstu.py'
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-quick}
mkdir -p gpurun_out/$TAG
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/test.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/$TAG/test.log | tail -30; tail -5 gpurun_out/$TAG/test.log; exit 1; }
  tail -1 gpurun_out/$TAG/test.log
fi
timeout -k 10 400 python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/$TAG/bench.log 2>&1 \
  || { tail -20 gpurun_out/$TAG/bench.log; exit 1; }
tail -1 gpurun_out/$TAG/bench.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('C2', d['value'], d['ms_per_step'], d['roofline']['per_step_device_ms'])
print('step_hbm', d['roofline'].get('step_hbm'))
print('cpu', d.get('cpu_baseline'))
if d.get('c2_two_blocks'): print('c2_two_blocks', d['c2_two_blocks']['value'], d['c2_two_blocks']['ms_per_step'])
for k in ('c3','c3_bf16','c2_bf16','e2e_train_step','c5_train_step'):
    if d.get(k): print(k, d[k].get('value'), d[k].get('ms_per_step'), d[k].get('per_step_device_ms',''))
r=d.get('retrieval');
if r: print('C4', r['ms_per_query_batch'], r['per_query_batch_device_ms'])
"
