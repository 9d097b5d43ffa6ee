#!/bin/bash
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_runner.py -x -q -s --timeout 200 --timeout-method thread > gpurun_out/r2s_tests.log 2>&1
