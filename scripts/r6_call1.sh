#!/bin/bash
# Round-6 GPU call: OOB probe, smoke, GPU suite (failures reported, not fatal), headline
# profile, attn_bwd_dkv counters.  Any crash / timeout (exit >= 124) ends the call.
set -o pipefail
TAG=${1:-r6a}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
fatal() { [ "$1" -ge 124 ] && { echo "FATAL rc=$1 at $2"; exit 1; }; return 0; }
timeout -k 10 60 ./scripts/probe/oob_probe > gpurun_out/$TAG/probe.log 2>&1; rc=$?
tail -2 gpurun_out/$TAG/probe.log; fatal $rc probe; [ $rc -ne 0 ] && exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" \
  > gpurun_out/$TAG/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/$TAG/smoke.log; fatal $rc smoke
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_a16.py -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/$TAG/test_a16.log 2>&1; rc=$?; tail -3 gpurun_out/$TAG/test_a16.log; fatal $rc a16tests
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_a16.py > gpurun_out/$TAG/test.log 2>&1; rc=$?; tail -3 gpurun_out/$TAG/test.log; fatal $rc tests
[ "${SKIP_PROF:-0}" = 1 ] && { echo CALL DONE; exit 0; }
bash scripts/profile_round.sh ${TAG}_head "--steps 20 --warmup 5 --no-cpu-baseline --retrieval-steps 5 --e2e-steps 0 --sweep= --c3-steps 0 --no-bf16-leg --c5-steps 0" || exit 1
grep '"metric"' gpurun_out/${TAG}_head/bench_trace.log > gpurun_out/${TAG}_head/bench_line.json || true
bash scripts/attn_counters.sh ${TAG}_dkv128 c2 "--hepi --only bwd" || exit 1
bash scripts/attn_counters.sh ${TAG}_dkv2048 c2 "--hepi --only bwd --batch 2048" || exit 1
echo CALL DONE
