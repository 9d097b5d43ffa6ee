#!/bin/bash
# attention backward workgroup timelines (diagnostic stamp build)
set -e
cd $GRAFT_REPO_ROOT
export GR_HSTU_LIB=vlib/libgr_stamp.so
for args in "--batch 128" "--batch 128 --split" "--batch 32" "--batch 512" "--batch 128 --nobias"; do
  timeout -k 5 90 python scripts/timeline_bwd.py $args >> gpurun_out/r2n_tl.jsonl
done
