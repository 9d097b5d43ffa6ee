#!/bin/bash
# a16 tests + HSTU bf16 tests, C3 bf16 A/B, then a kernel trace and the FETCH / WRITE passes
# of the a16 C3 step (per-kernel HBM bytes).
set -o pipefail
TAG=${1:-r6d}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_a16.py tests/test_gpu_hstu.py ${EXTRA_TESTS:-} -k "${TEST_K:-a16 or bf16}" -m gpu -q \
  --timeout 300 --timeout-method thread > gpurun_out/$TAG/test.log 2>&1; rc=$?
tail -4 gpurun_out/$TAG/test.log; [ $rc -ge 124 ] && exit 1
timeout -k 10 300 python3 -u scripts/c3_ab.py --steps 5 > gpurun_out/$TAG/c3_ab.jsonl 2>&1 || { tail -20 gpurun_out/$TAG/c3_ab.jsonl; exit 1; }
cut -c1-300 gpurun_out/$TAG/c3_ab.jsonl
[ "${PROF:-1}" = 1 ] || { echo CALL DONE; exit 0; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/trace -o run --output-format csv -- \
  python3 scripts/c3_ab.py --only a16 --steps 3 > gpurun_out/$TAG/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/$TAG/fetch -o run --output-format csv -- \
  python3 scripts/c3_ab.py --only a16 --steps 3 > gpurun_out/$TAG/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/$TAG/write -o run --output-format csv -- \
  python3 scripts/c3_ab.py --only a16 --steps 3 > gpurun_out/$TAG/write.log 2>&1 || exit 1
echo CALL DONE
