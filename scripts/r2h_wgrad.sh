set -e
cd $GRAFT_REPO_ROOT
for r in 0 64 128 256 512 1024; do
  if [ $r -gt 0 ]; then export GR_WGRAD_RPS=$r; fi
  echo "rps=$r $(timeout -k 5 60 python scripts/gemm_micro.py --shape c2 --wgrad-only --iters 30)" >> gpurun_out/r2h_wgrad.txt
done
unset GR_WGRAD_RPS
echo "full $(timeout -k 5 60 python scripts/gemm_micro.py --shape c2 --iters 30)" >> gpurun_out/r2h_wgrad.txt
