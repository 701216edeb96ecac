#!/bin/bash
# rocprofv3 kernel-stats of the C2 bench (graph replay), summarised per step: tools/step_profile.sh <outdir>
out=${1:-gpurun_out/sp}
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-hbm-line > $out.log 2>&1
