#!/bin/bash
# A/B of mips_topk at C4 shapes over prebuilt libraries (ab/libgr_<name>.so), interleaved:
#   gpurun -- 'bash scripts/topk_ab.sh "base new" [topk_micro args]'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/tab
names=$1; shift
for r in 1 2; do
  for n in $names; do
    GR_HSTU_LIB=$PWD/ab/libgr_$n.so timeout -k 10 120 python scripts/topk_micro.py "$@" > gpurun_out/tab/${n}_$r.txt 2>&1 || exit 1
    echo "== $n $r"; grep -E "ms/batch|candidates|mips_" gpurun_out/tab/${n}_$r.txt
  done
done
