#!/bin/bash
# bench.py A/B on one box, interleaved: --adamw flat vs torch (every leg), twice.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r6p}
mkdir -p gpurun_out/$TAG
for rep in 1 2; do
  for a in flat torch; do
    timeout -k 10 400 python3 -u bench.py --adamw $a --no-cpu-baseline > gpurun_out/$TAG/bench_${a}_$rep.log 2>&1 || { tail -20 gpurun_out/$TAG/bench_${a}_$rep.log; exit 1; }
    tail -1 gpurun_out/$TAG/bench_${a}_$rep.log > gpurun_out/$TAG/bench_${a}_$rep.json
    python3 -c "
import json; d=json.load(open('gpurun_out/$TAG/bench_${a}_$rep.json'))
print('$a', $rep, d['value'], d['c3_bf16']['value'], d['c3']['value'], d['c2_bf16']['value'], d['c2_two_blocks']['value'], d['e2e_train_step']['value'], d['c5_train_step']['value'])"
  done
done
