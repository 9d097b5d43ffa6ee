#!/bin/bash
# r3ae: float4-staged bf16 row panel (GR_OPT_PANEL_VEC): bit-exact test, full GPU suite, default bench
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest tests/test_gpu_hstu.py -x -v -k "panel_vec or bf16_mode" --timeout 200 --timeout-method thread > gpurun_out/r3ae_vec.log 2>&1 || { tail -40 gpurun_out/r3ae_vec.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r3ae_vec.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3ae_test.log 2>&1 || { grep -E "FAIL|Error|error|rel err|assert" gpurun_out/r3ae_test.log | tail -30; tail -5 gpurun_out/r3ae_test.log; exit 1; }
tail -2 gpurun_out/r3ae_test.log
timeout -k 10 600 python -u bench.py > gpurun_out/r3ae_bench.log 2>&1 || { tail -20 gpurun_out/r3ae_bench.log; exit 1; }
python3 - <<'PY'
import json
t=open('gpurun_out/r3ae_bench.log').read(); i=t.find('{"metric'); p=json.loads(t[i:].splitlines()[0])
print('c2', p['value'], p['ms_per_step'], p['roofline'].get('frac'))
for k in ('c3','c3_bf16','c2_bf16'):
    v=p.get(k) or {}
    print(k, v.get('value'), v.get('ms_per_step'), v.get('per_step_device_ms'))
print('ret', p['retrieval']['ms_per_query_batch'])
PY
