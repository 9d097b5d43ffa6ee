#!/bin/bash
# GPU check on the box (run via gpurun): smoke(), then the GPU test suite (optionally a
# subset: pass pytest selectors as arguments).  Logs under gpurun_out/$TAG/.
#   gpurun -- 'TAG=r4a bash scripts/gpu_check.sh tests/test_gpu_distributed.py'
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-check}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" \
  > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
SEL=${*:-tests}
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/$TAG/test.log 2>&1 || { grep -E "FAIL|Error|error|rel err|assert" gpurun_out/$TAG/test.log | tail -30; tail -5 gpurun_out/$TAG/test.log; exit 1; }
tail -1 gpurun_out/$TAG/test.log
