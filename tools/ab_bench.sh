#!/bin/bash
# Same-box A/B of a tools-build switch on the C2 step: alternating runs, A = the environment assignment in $1
# (e.g. ESGPT_GEMM_TILE_FWD=11), B = the default.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  env $1 timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/ab_a.log 2>&1 || exit 1
  echo "A $1: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_a.log)"
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/ab_b.log 2>&1 || exit 1
  echo "B default: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_b.log)"
done
