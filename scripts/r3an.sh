#!/bin/bash
# r3an: final round-3 check at HEAD: smoke(), full GPU suite
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r3an_smoke.log 2>&1 || { tail -20 gpurun_out/r3an_smoke.log; exit 1; }
tail -1 gpurun_out/r3an_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3an_test.log 2>&1 || { grep -E "FAIL|Error|error|rel err|assert" gpurun_out/r3an_test.log | tail -30; tail -5 gpurun_out/r3an_test.log; exit 1; }
tail -1 gpurun_out/r3an_test.log
