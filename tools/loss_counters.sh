#!/bin/bash
# SQ counters of the C2 attention forward / backward (tools/loss_pmc.py, dropout 0.1), two passes + a kernel trace.
cd "$(dirname "$0")/.."
R=$(pwd); mkdir -p gpurun_out/loss_pmc
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/loss_pmc/trace -o run -- python3 tools/loss_pmc.py > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA -d $R/gpurun_out/loss_pmc/p1 -o run -- python3 tools/loss_pmc.py > /dev/null 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/loss_pmc/p2 -o run -- python3 tools/loss_pmc.py > /dev/null 2>&1 || exit 3
find gpurun_out/loss_pmc -name "*.csv" | head -20
