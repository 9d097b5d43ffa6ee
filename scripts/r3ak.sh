#!/bin/bash
# r3ak (late round 3, HEAD): full GPU suite, then the default bench
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3ak_test.log 2>&1 || { grep -E "FAIL|Error|error|rel err|assert" gpurun_out/r3ak_test.log | tail -30; tail -5 gpurun_out/r3ak_test.log; exit 1; }
tail -2 gpurun_out/r3ak_test.log
timeout -k 10 600 python -u bench.py > gpurun_out/r3ak_bench.log 2>&1 || { tail -20 gpurun_out/r3ak_bench.log; exit 1; }
grep '^{"metric' gpurun_out/r3ak_bench.log | cut -c1-600
