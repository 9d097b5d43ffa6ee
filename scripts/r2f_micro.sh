set -e
cd $GRAFT_REPO_ROOT
for B in 32 128 512; do
  timeout -k 5 60 python scripts/attn_micro.py --shape c2 --batch $B --hepi --iters 30 >> gpurun_out/r2f_micro.jsonl
  GR_ATTN_BWD_SPLIT=1 timeout -k 5 60 python scripts/attn_micro.py --shape c2 --batch $B --hepi --iters 30 >> gpurun_out/r2f_micro.jsonl
done
GR_ATTN_BWD_SPLIT=1 timeout -k 5 60 python scripts/attn_micro.py --shape c2 --batch 128 --hepi --nobias --iters 30 >> gpurun_out/r2f_micro.jsonl
