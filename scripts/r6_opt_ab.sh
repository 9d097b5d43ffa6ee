set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6o
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_next_rows.py tests/test_gpu_topk.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r6o/test.log 2>&1; rc=$?
tail -3 gpurun_out/r6o/test.log; [ $rc -ne 0 ] && exit 1
timeout -k 10 600 python3 -u scripts/opt_ab.py > gpurun_out/r6o/ab.jsonl 2>&1 || { tail -20 gpurun_out/r6o/ab.jsonl; exit 1; }
grep '^{' gpurun_out/r6o/ab.jsonl
