#!/bin/bash
# Same-box A/B on the C2 step (HBM-resident batches): optimizer host-launched (default) vs its own graph (--opt-graph)
set -o pipefail
mkdir -p gpurun_out
one() { timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-roofline $2 > gpurun_out/ab.log 2>&1 || exit 1
        python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); p=d['value_hbm_resident'] or {}; print('$1', d['ms_per_step'], d['ms_per_step_median'], 'hbm', p.get('ms_per_step'))"; }
for i in 1 2 3; do one default ""; one opt-graph "--opt-graph"; done
