#!/bin/bash
# r3h: counters of the C4 filter pass (10M x 50, B = 128)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=gpurun_out/r3h; mkdir -p $T
A="scripts/topk_micro.py --iters 3"
timeout -k 10 120 python3 scripts/topk_micro.py --iters 20 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM \
  -d $T/p1 -o run --output-format csv -- python3 $A > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE \
  -d $T/p2 -o run --output-format csv -- python3 $A > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TD_BUSY_avr \
  -d $T/p3 -o run --output-format csv -- python3 $A > /dev/null || true
python3 scripts/counter_summary.py $T | sed -n '/mips_filter_kernel<1, 2, 8, false>/,/WAVE_CYCLES/p'
