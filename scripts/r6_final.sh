#!/bin/bash
# Round-6 end evidence in one GPU call: smoke, the whole GPU suite, the default bench line,
# the headline profile (C2 + C4 legs: kernel trace, FETCH / WRITE passes) and the C3 bf16
# (a16) step profile.  Any crash / timeout (exit >= 124) ends the call.
set -o pipefail
TAG=${1:-r6final}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
fatal() { [ "$1" -ge 124 ] && { echo "FATAL rc=$1 at $2"; exit 1; }; return 0; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" \
  > gpurun_out/$TAG/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/$TAG/smoke.log; fatal $rc smoke; [ $rc -ne 0 ] && exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/$TAG/test.log 2>&1; rc=$?; tail -1 gpurun_out/$TAG/test.log; fatal $rc tests
timeout -k 10 600 python3 -u bench.py > gpurun_out/$TAG/bench.log 2>&1; rc=$?; fatal $rc bench; [ $rc -ne 0 ] && exit 1
tail -1 gpurun_out/$TAG/bench.log > gpurun_out/$TAG/bench.json
bash scripts/profile_round.sh ${TAG}_head "--steps 20 --warmup 5 --no-cpu-baseline --retrieval-steps 5 --e2e-steps 0 --sweep= --c3-steps 0 --no-bf16-leg --c5-steps 0" || exit 1
grep '"metric"' gpurun_out/${TAG}_head/bench_trace.log > gpurun_out/${TAG}_head/bench_line.json || true
D=gpurun_out/${TAG}_c3
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- \
  python3 scripts/c3_ab.py --only a16 --steps 3 > $D/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run --output-format csv -- \
  python3 scripts/c3_ab.py --only a16 --steps 3 > $D/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $D/write -o run --output-format csv -- \
  python3 scripts/c3_ab.py --only a16 --steps 3 > $D/write.log 2>&1 || exit 1
echo CALL DONE
