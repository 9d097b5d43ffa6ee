#!/bin/bash
# r3z: HSTU layer tests + headline-only bench (C2 step)
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u -m pytest tests/test_gpu_hstu.py tests/test_gpu_wgrad.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3z_test.log 2>&1 || { grep -E "FAIL|Error|error|rel err|assert" gpurun_out/r3z_test.log | tail -30; exit 1; }
tail -1 gpurun_out/r3z_test.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --c3-steps 0 --no-bf16-leg --e2e-steps 0 --c5-steps 0 --sweep= --retrieval-d256-items 0 > gpurun_out/r3z_bench.log 2>&1 || { tail -20 gpurun_out/r3z_bench.log; exit 1; }
python3 - <<'PY'
import json
t=open('gpurun_out/r3z_bench.log').read(); i=t.find('{"metric'); p=json.loads(t[i:].splitlines()[0])
print(p['value'], p['ms_per_step'], p['roofline']['per_step_device_ms'])
PY
