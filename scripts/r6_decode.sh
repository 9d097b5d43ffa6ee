#!/bin/bash
# Cached-decoding GPU tests, then the encoder tests that share STULayerFunction.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r6dec}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_decode.py > gpurun_out/$TAG/decode.log 2>&1 || { tail -60 gpurun_out/$TAG/decode.log; exit 1; }
tail -15 gpurun_out/$TAG/decode.log
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_hstu.py tests/test_gpu_a16.py > gpurun_out/$TAG/hstu.log 2>&1 || { tail -40 gpurun_out/$TAG/hstu.log; exit 1; }
tail -3 gpurun_out/$TAG/hstu.log
