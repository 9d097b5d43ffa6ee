#!/bin/bash
# the driver's default bench invocation, timed
set -e
cd $GRAFT_REPO_ROOT
start=$(date +%s)
timeout -k 10 900 python bench.py > gpurun_out/r2ab_bench.json 2> gpurun_out/r2ab_bench.err
echo "elapsed $(( $(date +%s) - start )) s" > gpurun_out/r2ab_time.txt
