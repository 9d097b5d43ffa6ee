set -e
cd $GRAFT_REPO_ROOT
for B in 32 128 512; do
  timeout -k 5 60 python scripts/attn_micro.py --split --shape c2 --batch $B --hepi --iters 30 >> gpurun_out/r2f_micro.jsonl
  timeout -k 5 60 python scripts/attn_micro.py --shape c2 --batch $B --hepi --iters 30 >> gpurun_out/r2f_micro.jsonl
done
timeout -k 5 60 python scripts/attn_micro.py --split --shape c2 --batch 128 --hepi --nobias --iters 30 >> gpurun_out/r2f_micro.jsonl
