#!/bin/bash
# a16 tests + the HSTU bf16 tests, then the C3 bf16 A/B (bf16 activations on / off).
set -o pipefail
TAG=${1:-r6b}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_a16.py tests/test_gpu_hstu.py -k "a16 or bf16" -m gpu -q \
  --timeout 300 --timeout-method thread > gpurun_out/$TAG/test.log 2>&1; rc=$?
tail -4 gpurun_out/$TAG/test.log; [ $rc -ge 124 ] && exit 1
timeout -k 10 300 python3 -u scripts/c3_ab.py --steps 5 > gpurun_out/$TAG/c3_ab.jsonl 2>&1 || { tail -20 gpurun_out/$TAG/c3_ab.jsonl; exit 1; }
cut -c1-300 gpurun_out/$TAG/c3_ab.jsonl
echo CALL DONE
