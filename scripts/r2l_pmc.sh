set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2l
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_MFMA"
timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/r2l/attn -o run --output-format csv -- python3 scripts/attn_micro.py --shape c2 --only bwd --hepi --iters 5 > gpurun_out/r2l/attn.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/r2l/wg -o run --output-format csv -- python3 scripts/gemm_micro.py --shape c2 --wgrad-only --iters 5 > gpurun_out/r2l/wg.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/r2l/fwd -o run --output-format csv -- python3 scripts/attn_micro.py --shape c2 --only fwd --iters 5 > gpurun_out/r2l/fwd.log 2>&1
echo done
