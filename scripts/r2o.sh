#!/bin/bash
set -e
cd $GRAFT_REPO_ROOT
export GR_HSTU_LIB=vlib/libgr_stamp.so
for B in 32 128; do
  echo "B=$B" >> gpurun_out/r2o_stamp.txt
  timeout -k 5 90 python scripts/stamp_dkv.py --batch $B --len 200 --hepi >> gpurun_out/r2o_stamp.txt
done
