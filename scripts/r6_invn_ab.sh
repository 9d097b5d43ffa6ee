#!/bin/bash
# A/B of the wide bf16 attention with 1/N folded into the epilogues (libgr_hstu.so) vs the
# previous build (libgr_hstu_old.so): C3-shape micro, interleaved, then the bf16 tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r6invn}
mkdir -p gpurun_out/$TAG
OLD=$PWD/mygenerativerecommenders_amd/libgr_hstu_old.so
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export GR_HSTU_LIB=$OLD; else unset GR_HSTU_LIB; fi
    timeout -k 10 240 python3 -u scripts/attn_micro.py --shape c3 --bf16 --hepi > gpurun_out/$TAG/micro_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/$TAG/micro_${v}_$rep.log; exit 1; }
    echo "== $v $rep"; tail -4 gpurun_out/$TAG/micro_${v}_$rep.log
  done
done
unset GR_HSTU_LIB
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_attention.py tests/test_gpu_a16.py tests/test_gpu_hstu.py -k "bf16 or a16" \
  > gpurun_out/$TAG/tests.log 2>&1; rc=$?
tail -5 gpurun_out/$TAG/tests.log
exit $rc
