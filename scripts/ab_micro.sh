#!/bin/bash
# A/B a micro-benchmark over prebuilt libraries (ab/libgr_<name>.so), interleaved, twice:
#   gpurun -- 'bash scripts/ab_micro.sh "base mf" scripts/attn_micro.py --shape c3 --bf16'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
names=$1; shift
for rep in 1 2; do
  for n in $names; do
    out=$(GR_HSTU_LIB=$PWD/ab/libgr_$n.so timeout -k 10 120 python "$@" 2>/dev/null | tail -1) || exit 1
    echo "$n $out"
  done
done
