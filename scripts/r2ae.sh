#!/bin/bash
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_embeddings.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2ae_tests.log 2>&1
