#!/bin/bash
# Grouped projection backward at the C2 shapes over staging form x dX tile x dW tile (tools build).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for g in 0 2 3; do for x in 11 21 22; do for w in 11 22; do
  echo "== BWD_GLDS=$g TILE_DX=$x TILE_DW=$w"
  ESGPT_GEMM_BWD_GLDS=$g ESGPT_GEMM_TILE_DX=$x ESGPT_GEMM_TILE_DW=$w timeout -k 10 60 \
    bash tools/with_tuning.sh python -u tools/bwd_pair_time.py 2>&1 | grep -v amdgpu.ids || exit 1
done; done; done 2>&1 | tee gpurun_out/glds_bwd_sweep.log
