#!/bin/bash
# bf16 dkv private dpos histograms: parity + C2/C3 micro + encoder bench legs
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_hstu.py -x -q -s -k "bf16 or concat or golden" --timeout 200 --timeout-method thread > gpurun_out/r2m_tests.log 2>&1
for sh in c2 c3; do
  timeout -k 5 90 python scripts/attn_micro.py --shape $sh --only bwd --hepi --iters 10 --bf16 >> gpurun_out/r2m_micro.jsonl
done
timeout -k 10 300 python bench.py --no-retrieval-leg --no-cpu-baseline --e2e-steps 0 --sweep "" > gpurun_out/r2m_bench.json 2> gpurun_out/r2m_bench.err
