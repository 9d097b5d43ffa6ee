set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -x -q -s -k bf16 --timeout 200 --timeout-method thread > gpurun_out/r2j_tests.log 2>&1
for sh in c2 c3; do
  timeout -k 5 90 python scripts/attn_micro.py --shape $sh --only fwd --iters 20 >> gpurun_out/r2j_micro.jsonl
  timeout -k 5 90 python scripts/attn_micro.py --shape $sh --only fwd --iters 20 --bf16 >> gpurun_out/r2j_micro.jsonl
done
