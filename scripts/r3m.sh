#!/bin/bash
# r3m: C3 legs (fp32 and bf16) with per-kernel device time
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --sweep "" --no-retrieval-leg --e2e-steps 0 --c5-steps 0 --no-bf16-leg --c3-steps 5 > gpurun_out/r3m_bench.log 2>&1 || { tail -20 gpurun_out/r3m_bench.log; exit 1; }
python3 - <<'PY'
import json
t=open('gpurun_out/r3m_bench.log').read(); i=t.find('{"metric'); p=json.loads(t[i:].splitlines()[0])
for k in ('c3','c3_bf16'):
    r=p[k]; print(k, r['value'], r['ms_per_step'], r['roofline']['frac'], json.dumps(r['per_step_device_ms']))
PY
