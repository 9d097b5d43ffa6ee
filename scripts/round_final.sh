#!/bin/bash
# End-of-round evidence on the GPU box (run via gpurun), in two calls:
#   gpurun -- 'bash scripts/round_final.sh check TAG'    smoke + the whole GPU suite + default bench
#   gpurun -- 'bash scripts/round_final.sh profile TAG'  rocprofv3 trace + FETCH/WRITE passes
# Outputs under gpurun_out/TAG/; then python scripts/pmc_summary.py gpurun_out/TAG TAG
set -o pipefail
MODE=${1:-check}
TAG=${2:-final}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
if [ "$MODE" = check ]; then
  timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" \
    > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
  tail -1 gpurun_out/$TAG/smoke.log
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/test.log 2>&1 || { tail -30 gpurun_out/$TAG/test.log; exit 1; }
  tail -1 gpurun_out/$TAG/test.log
  timeout -k 10 600 python3 -u bench.py > gpurun_out/$TAG/bench.log 2>&1 || { tail -20 gpurun_out/$TAG/bench.log; exit 1; }
  tail -1 gpurun_out/$TAG/bench.log > gpurun_out/$TAG/bench.json
  python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
else
  bash scripts/profile_round.sh $TAG
fi
