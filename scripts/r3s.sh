#!/bin/bash
# r3s: counters of the f32 attention backward at C2 (split launches: dK/dV, dQ), B = 128 and 512
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for B in 128 512; do
T=gpurun_out/r3s_b$B; mkdir -p $T
A="scripts/attn_micro.py --shape c2 --only bwd --hepi --split --batch $B --iters 3"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM \
  -d $T/p1 -o run --output-format csv -- python3 $A > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE \
  -d $T/p2 -o run --output-format csv -- python3 $A > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_IFETCH SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU \
  -d $T/p3 -o run --output-format csv -- python3 $A > /dev/null || true
echo "== B=$B"; python3 scripts/counter_summary.py $T
done
