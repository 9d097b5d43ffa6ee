#!/bin/bash
# r3i: C3 attention kernels (d = 256, L = 2048, B = 32): fp32 / bf16, with / without bias
set -o pipefail
cd "$(dirname "$0")/.."
run() { timeout -k 10 200 python -u scripts/attn_micro.py --shape c3 --hepi --iters 5 "$@" | python3 -c "import json,sys; d=json.load(sys.stdin); print('$*', {k: (v['avg_us'], v['tflops']) for k, v in d['kernels'].items()})" || exit 1; }
run
run --nobias
run --bf16
run --bf16 --nobias
