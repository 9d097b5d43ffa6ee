#!/bin/bash
# r3k: wide bf16 backward ablations (vlib/libgr_abl{4..7}: no dts / no dpos / neither / branch-free dts),
# one accumulator tile), C3 shape
set -o pipefail
cd "$(dirname "$0")/.."
run() { timeout -k 10 120 python -u scripts/attn_micro.py --shape c3 --bf16 --only bwd --iters 10 "$@"; }
{ echo base; run; echo nobias; run --nobias;
  for n in 4 5 6 7; do echo abl$n; GR_HSTU_LIB=vlib/libgr_abl$n.so run; done; } > gpurun_out/r3k.log 2>&1 || { tail -20 gpurun_out/r3k.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3k.log
