#!/bin/bash
# r3aj: wide outputs split into two column panels when the row grid is under two blocks per
# CU (C2 ln_uvqk_fwd: 400 blocks on 256 CUs); HSTU tests, C2 micro, C2 / C3 bench legs
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest tests/test_gpu_hstu.py tests/test_gpu_runner.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3aj_test.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/r3aj_test.log | tail -30; tail -3 gpurun_out/r3aj_test.log; exit 1; }
tail -1 gpurun_out/r3aj_test.log
for f in "" "--bf16-panels"; do
timeout -k 10 120 python -u scripts/gemm_micro.py --shape c2 --iters 50 $f > gpurun_out/r3aj_micro.log 2>&1 || { tail -20 gpurun_out/r3aj_micro.log; exit 1; }
tail -1 gpurun_out/r3aj_micro.log
done
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-retrieval-leg --e2e-steps 0 --c5-steps 0 --sweep= --c3-steps 0 > gpurun_out/r3aj_bench.log 2>&1 || { tail -20 gpurun_out/r3aj_bench.log; exit 1; }
python3 - <<'PY'
import json
t=open('gpurun_out/r3aj_bench.log').read(); i=t.find('{"metric'); p=json.loads(t[i:].splitlines()[0])
print('c2', p['value'], p['ms_per_step'], p['roofline'].get('frac'), p['roofline'].get('per_step_device_ms'))
v=p.get('c2_bf16') or {}
print('c2_bf16', v.get('value'), v.get('ms_per_step'))
PY
