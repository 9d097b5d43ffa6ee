#!/bin/bash
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2x_tests.log 2>&1
