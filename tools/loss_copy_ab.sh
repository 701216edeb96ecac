#!/bin/bash
# Same-box A/B on the C2 step: the replayed step's loss copy riding in the optimizer's prepare launch (default) vs
# its own pack launch (bench.py --loss-pack), alternating runs.
set -o pipefail
mkdir -p gpurun_out
one() { timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-roofline $2 > gpurun_out/ab.log 2>&1 || exit 1
        echo "$1: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log) $(grep -o '"ms_per_step_median": [0-9.]*' gpurun_out/ab.log)"; }
for i in 1 2 3; do one in-opt ""; one pack "--loss-pack"; done
