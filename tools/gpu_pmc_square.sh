set -o pipefail
mkdir -p gpurun_out/pmc_sq
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_sq/kt -o kt -- python tools/gemm_square.py > gpurun_out/pmc_sq/kt.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/pmc_sq/p1 -o p1 -- python tools/gemm_square.py > gpurun_out/pmc_sq/p1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq/p2 -o p2 -- python tools/gemm_square.py > gpurun_out/pmc_sq/p2.log 2>&1
rc=$?; echo rc=$rc; find gpurun_out/pmc_sq -name "*.csv" | head; exit $rc
