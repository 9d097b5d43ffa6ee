#!/bin/bash
# Counter passes for the attention micro-benchmark (run via gpurun).
#   bash scripts/attn_counters.sh TAG SHAPE ["--bf16 --hepi --only bwd"]
set -e
TAG=${1:-attn}
SHAPE=${2:-c2}
EXTRA=${3:-}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
timeout -k 10 200 python3 scripts/attn_micro.py --shape $SHAPE $EXTRA --iters 20 > gpurun_out/$TAG/micro.json
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU \
  -d gpurun_out/$TAG/p1 -o run --output-format csv -- python3 scripts/attn_micro.py --shape $SHAPE $EXTRA --iters 5 > /dev/null
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM \
  -d gpurun_out/$TAG/p2 -o run --output-format csv -- python3 scripts/attn_micro.py --shape $SHAPE $EXTRA --iters 5 > /dev/null || true
echo counters done
