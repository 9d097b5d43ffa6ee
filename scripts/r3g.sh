#!/bin/bash
# r3g: bf16 filter copy at 4-dim padding: parity + C4 retrieval timing
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u -m pytest tests/test_gpu_topk.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3g_test.log 2>&1 || { tail -30 gpurun_out/r3g_test.log; exit 1; }
tail -2 gpurun_out/r3g_test.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --sweep "" --c3-steps 0 --no-bf16-leg --e2e-steps 0 --c5-steps 0 > gpurun_out/r3g_bench.log 2>&1 || { tail -20 gpurun_out/r3g_bench.log; exit 1; }
python3 - <<'PY'
import json
t=open('gpurun_out/r3g_bench.log').read(); i=t.find('{"metric'); p=json.loads(t[i:].splitlines()[0])
r=p['retrieval']; print(p['value'], r['value'], r['ms_per_query_batch'], r['per_query_batch_device_ms'], r['check']['ok'], r['roofline']['achieved'], r['roofline']['frac'])
PY
