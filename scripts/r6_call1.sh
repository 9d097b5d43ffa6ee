#!/bin/bash
# Round-6 first GPU call: OOB probe, smoke + GPU suite, headline profile, attn_bwd_dkv counters.
set -o pipefail
TAG=${1:-r6a}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
timeout -k 10 60 ./scripts/probe/oob_probe > gpurun_out/$TAG/probe.log 2>&1 || { cat gpurun_out/$TAG/probe.log; exit 1; }
tail -2 gpurun_out/$TAG/probe.log
bash scripts/round_check.sh $TAG || exit 1
bash scripts/profile_round.sh ${TAG}_head "--steps 20 --warmup 5 --no-cpu-baseline --retrieval-steps 5 --e2e-steps 0 --sweep= --c3-steps 0 --no-bf16-leg --c5-steps 0" || exit 1
grep '"metric"' gpurun_out/${TAG}_head/bench_trace.log > gpurun_out/${TAG}_head/bench_line.json || true
bash scripts/attn_counters.sh ${TAG}_dkv128 c2 "--hepi --only bwd" || exit 1
bash scripts/attn_counters.sh ${TAG}_dkv2048 c2 "--hepi --only bwd --batch 2048" || exit 1
echo CALL DONE
