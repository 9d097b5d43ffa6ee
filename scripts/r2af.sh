#!/bin/bash
# full GPU suite + smoke + default bench on the current tree
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2af_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2af_smoke.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/r2af_bench.json 2> gpurun_out/r2af_bench.err
