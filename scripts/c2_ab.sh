set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/c2ab
for rep in 1 2 3; do for n in old new; do
  GR_HSTU_LIB=$PWD/ab/libgr_$n.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-retrieval-leg --e2e-steps 0 --sweep "" --c3-steps 0 --no-bf16-leg --c5-steps 0 > gpurun_out/c2ab/run.log 2>&1 || { tail -20 gpurun_out/c2ab/run.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/c2ab/run.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
