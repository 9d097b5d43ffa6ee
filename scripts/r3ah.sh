#!/bin/bash
# r3ah: float4 staging on the backward panels only; HSTU tests, C2 / C3 bench legs, then the
# round-3 profiles (headline C2 + C4; C3 fp32 + bf16): kernel trace + FETCH / WRITE passes
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest tests/test_gpu_hstu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3ah_test.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/r3ah_test.log | tail -30; tail -3 gpurun_out/r3ah_test.log; exit 1; }
tail -1 gpurun_out/r3ah_test.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-retrieval-leg --e2e-steps 0 --c5-steps 0 --sweep= --c3-steps 5 > gpurun_out/r3ah_bench.log 2>&1 || { tail -20 gpurun_out/r3ah_bench.log; exit 1; }
python3 - <<'PY'
import json
t=open('gpurun_out/r3ah_bench.log').read(); i=t.find('{"metric'); p=json.loads(t[i:].splitlines()[0])
print('c2', p['value'], p['ms_per_step'], p['roofline'].get('frac'))
for k in ('c3','c3_bf16','c2_bf16'):
    v=p.get(k) or {}
    print(k, v.get('value'), v.get('ms_per_step'), v.get('per_step_device_ms'))
PY
bash scripts/profile_round.sh r3ah_h "--steps 20 --warmup 5 --no-cpu-baseline --retrieval-steps 5 --c3-steps 0 --no-bf16-leg --e2e-steps 0 --c5-steps 0 --sweep= --retrieval-d256-items 0" || exit 1
bash scripts/profile_round.sh r3ah_c3 "--steps 2 --warmup 1 --no-cpu-baseline --no-retrieval-leg --c3-steps 3 --e2e-steps 0 --c5-steps 0 --sweep=" || exit 1
grep '^{"metric' gpurun_out/r3ah_h/bench_trace.log | cut -c1-200
