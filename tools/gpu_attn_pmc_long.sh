# SQ counters of the long-shape attention forward (B=4, L=4096, H=8, causal) for the parity form and the wide
# form (tools build, ESGPT_ATTN_FWD_NW), two counter passes each + a kernel trace.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd); export TMPDIR=/tmp ATTN_SHAPE=long
D="$R/eventstreamgpt_amd/tuning"
export ESGPT_AMD_LIB="$D/libesgpt_amd.so" ESGPT_AMD_TORCH_LIB="$D/libesgpt_torch.so"
for nw in 0 4; do
  export ESGPT_ATTN_FWD_NW=$nw
  O=$R/gpurun_out/attn_pmc_long/nw$nw; mkdir -p $O
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 tools/attn_pmc.py 0.0 > /dev/null 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA -d $O/p1 -o run -- python3 tools/attn_pmc.py 0.0 > /dev/null 2>&1 || exit 2
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/p2 -o run -- python3 tools/attn_pmc.py 0.0 > /dev/null 2>&1 || exit 3
  timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_FLAT SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_EXP SQ_ACTIVE_INST_SCA -d $O/p3 -o run -- python3 tools/attn_pmc.py 0.0 > /dev/null 2>&1 || echo "p3 failed (counter names)"
done
find gpurun_out/attn_pmc_long -name "*counter_collection.csv" | head
