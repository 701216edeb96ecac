#!/bin/bash
# Grouped projection backward at the C2 shapes under several fixed dW work-item targets (tools build).
for t in 0 256 512 1024; do
  echo "== ESGPT_GEMM_DW_TARGET=$t"; ESGPT_GEMM_DW_TARGET=$t timeout -k 10 100 python tools/bwd_pair_time.py 2>&1 | grep -v amdgpu || exit 1
done
