#!/bin/bash
# SQ counter passes for a micro-benchmark (run via gpurun):
#   bash scripts/counters.sh TAG scripts/gemm_micro.py --shape c2 --iters 5
set -e
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU \
  -d gpurun_out/$TAG/p1 -o run --output-format csv -- python3 "$@" > /dev/null
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM \
  -d gpurun_out/$TAG/p2 -o run --output-format csv -- python3 "$@" > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/t -o run --output-format csv -- python3 "$@" > /dev/null
echo counters done
