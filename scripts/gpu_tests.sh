#!/bin/bash
# Selected GPU tests then (optionally) the C2 sweep:  gpurun -- 'TAG=x bash scripts/gpu_tests.sh tests/a.py tests/b.py'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-tests}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/$TAG/test.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/$TAG/test.log | tail -30; tail -5 gpurun_out/$TAG/test.log; exit 1; }
tail -1 gpurun_out/$TAG/test.log
