#!/bin/bash
# r3ag: streamed LN-backward epilogue; 2- vs 3-wave form (GR_OPT_PANEL_VEC 1 / 2) at C3 bf16
set -o pipefail
cd "$(dirname "$0")/.."
#timeout -k 10 300 python -u -m pytest tests/test_gpu_hstu.py -x -q -k "panel_vec or bf16_mode" --timeout 200 --timeout-method thread > gpurun_out/r3ag_test.log 2>&1 || { tail -30 gpurun_out/r3ag_test.log; exit 1; }
#tail -1 gpurun_out/r3ag_test.log
for v in 0 1 2; do
  timeout -k 10 120 python -u scripts/gemm_micro.py --shape c3 --iters 20 --bf16-panels --panel-vec $v > gpurun_out/r3ag_micro_$v.log 2>&1 || { tail -20 gpurun_out/r3ag_micro_$v.log; exit 1; }
  tail -1 gpurun_out/r3ag_micro_$v.log
done
