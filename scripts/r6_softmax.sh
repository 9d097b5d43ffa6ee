#!/bin/bash
# softmax_rel_bias GPU tests, then the decode and encoder tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r6sm}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_softmax.py > gpurun_out/$TAG/softmax.log 2>&1 || { tail -60 gpurun_out/$TAG/softmax.log; exit 1; }
tail -15 gpurun_out/$TAG/softmax.log
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_decode.py tests/test_gpu_hstu.py tests/test_gpu_rel_bias.py > gpurun_out/$TAG/rest.log 2>&1 || { tail -40 gpurun_out/$TAG/rest.log; exit 1; }
tail -3 gpurun_out/$TAG/rest.log
