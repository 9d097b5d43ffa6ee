#!/bin/bash
# r3r: f32 attention backward at C2 -- LDS-read ablations (W_ABL 1: A operands as b128,
# 2: B operands as b128, 4: no bias clamps, 7: all; timing only, results wrong)
set -o pipefail
cd "$(dirname "$0")/.."
run() { timeout -k 10 90 python -u scripts/attn_micro.py --shape c2 --only bwd --hepi --iters 30 "$@" 2>&1 | grep -v amdgpu.ids; }
{ echo base; run; for n in 1 2 4 7; do echo abl$n; GR_HSTU_LIB=vlib/libgr_abl$n.so run; done; echo split; run --split; } > gpurun_out/r3r.log 2>&1 || { tail -20 gpurun_out/r3r.log; exit 1; }
cat gpurun_out/r3r.log
