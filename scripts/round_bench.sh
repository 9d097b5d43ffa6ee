#!/bin/bash
# The default bench.py run on the GPU box with its progress lines under gpurun_out/TAG/.
set -o pipefail
TAG=${1:-final}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python3 -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err \
  || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
grep "^\[bench" gpurun_out/$TAG/bench.err | tail -20
python3 -c "import json; d=json.loads(open('gpurun_out/$TAG/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d.get('cpu_baseline'))"
