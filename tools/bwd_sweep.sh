#!/bin/bash
# Grouped projection backward at the C2 shapes, whole and in parts (tools build: ESGPT_GEMM_DBG bits).
for d in 0 1 2 3 4 8; do
  echo "== ESGPT_GEMM_DBG=$d"; ESGPT_GEMM_DBG=$d timeout -k 10 100 python tools/bwd_pair_time.py 2>&1 | grep -v amdgpu || exit 1
done
