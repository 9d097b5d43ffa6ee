#!/bin/bash
# r3q: D > 64 filter path (top-k tests), concat_ua at any width (HSTU tests), retrieval legs
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 500 python -u -m pytest tests/test_gpu_topk.py tests/test_gpu_hstu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r3q_test.log 2>&1 || { grep -E "PASS|FAIL|Error|error" gpurun_out/r3q_test.log | tail -30; exit 1; }
grep -E "passed|failed" gpurun_out/r3q_test.log | tail -2
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --sweep "" --c3-steps 0 --no-bf16-leg --e2e-steps 0 --c5-steps 0 > gpurun_out/r3q_bench.log 2>&1 || { tail -20 gpurun_out/r3q_bench.log; exit 1; }
python3 - <<'PY'
import json
t=open('gpurun_out/r3q_bench.log').read(); i=t.find('{"metric'); p=json.loads(t[i:].splitlines()[0])
for k in ('retrieval','retrieval_d256'):
    r=p[k]; print(k, r['value'], r['ms_per_query_batch'], r['check'], r['per_query_batch_device_ms'], r['roofline']['frac'])
PY
