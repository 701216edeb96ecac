#!/bin/bash
# Per-section cost of event_stream_kernel at C2 (tools build, ESGPT_LOSS_SKIP bits: 1 pass-1 MULTI math, 2 pass-2
# terms, 4 subjects_with_events, 8 in-row TTE, 16 narrow-chunk store): kernel trace + SQ instruction counts per setting.
cd "$(dirname "$0")/.."
R=$(pwd); mkdir -p gpurun_out/loss_sec
export TMPDIR=/tmp
D=$R/eventstreamgpt_amd/tuning
export ESGPT_AMD_LIB="$D/libesgpt_amd.so" ESGPT_AMD_TORCH_LIB="$D/libesgpt_torch.so"
for s in ${SKIPS:-0 1 2 4 8 16 31}; do
  export ESGPT_LOSS_SKIP=$s
  timeout -s KILL 90 rocprofv3 --kernel-trace -d $R/gpurun_out/loss_sec/t$s -o run -- python3 tools/loss_pmc.py > /dev/null 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY -d $R/gpurun_out/loss_sec/p$s -o run -- python3 tools/loss_pmc.py > /dev/null 2>&1 || exit 2
  echo "skip $s done"
done
python3 tools/loss_sec_summary.py ${SKIPS:-0 1 2 4 8 16 31} | tee gpurun_out/loss_sec/summary.txt
find gpurun_out/loss_sec -name "*.db" -delete
