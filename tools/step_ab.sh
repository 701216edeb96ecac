#!/bin/bash
# Same-box A/B of a config's step (CONFIG, default C2; STEPS, default 200): product library vs the tools build (another revision of a kernel source), alternating
# 200-step runs (HBM-resident batches)
set -o pipefail
mkdir -p gpurun_out
one() { timeout -k 10 200 $2 python bench.py --config ${CONFIG:-C2} --steps ${STEPS:-200} --warmup 10 --dtype ${DTYPE:-bf16} --no-cpu-baseline --no-roofline --no-hbm-line > gpurun_out/sab.log 2>&1 || exit 1
        python -c "import json; d=json.loads(open('gpurun_out/sab.log').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['ms_per_step_median'])"; }
for i in 1 2 3; do one product ""; one tools "bash tools/with_tuning.sh"; done
