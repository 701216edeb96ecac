#!/bin/bash
# Loss-kernel parity tests + kernel trace of the C2 output loss (tools/loss_pmc.py).
cd "$(dirname "$0")/.."
R=$(pwd); mkdir -p gpurun_out/loss_chk
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_loss_paths_gpu.py \
  tests/test_gpu_parity.py -k "loss or golden or Loss" > gpurun_out/loss_chk/pytest.log 2>&1 || { tail -30 gpurun_out/loss_chk/pytest.log; exit 1; }
tail -3 gpurun_out/loss_chk/pytest.log
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/loss_chk/trace -o run -- python3 tools/loss_pmc.py > /dev/null 2>&1 || exit 2
f=$(find gpurun_out/loss_chk/trace -name "*kernel_stats.csv" | head -1); cat "$f" | cut -d, -f1-5 | head -20
