#!/bin/bash
# r3am: bf16 copies, 4 chunks per thread (loads first): attention + HSTU bf16 tests, C3 bench legs
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_hstu.py -x -q -k "bf16" --timeout 200 --timeout-method thread > gpurun_out/r3am_test.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/r3am_test.log | tail -30; tail -3 gpurun_out/r3am_test.log; exit 1; }
tail -1 gpurun_out/r3am_test.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-retrieval-leg --e2e-steps 0 --c5-steps 0 --sweep= --c3-steps 5 > gpurun_out/r3am_bench.log 2>&1 || { tail -20 gpurun_out/r3am_bench.log; exit 1; }
python3 - <<'PY'
import json
t=open('gpurun_out/r3am_bench.log').read(); i=t.find('{"metric'); p=json.loads(t[i:].splitlines()[0])
print('c2', p['value'], p['ms_per_step'])
for k in ('c3','c3_bf16','c2_bf16'):
    v=p.get(k) or {}
    print(k, v.get('value'), v.get('ms_per_step'), (v.get('per_step_device_ms') or {}).get('attn_bf16_copies'))
PY
