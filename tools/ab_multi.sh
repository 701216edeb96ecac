#!/bin/bash
# Same-box A/B of several tools-build switches on the C2 step (each: 2 alternating pairs against the default).
set -o pipefail
mkdir -p gpurun_out
one() { timeout -k 10 200 env $1 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/ab.log 2>&1 || exit 1
        echo "$1: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log)"; }
for sw in "$@"; do
  for i in 1 2; do one "$sw"; one "X=default"; done
done
