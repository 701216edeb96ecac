#!/bin/bash
# Same-box A/B of the C5 2 GiB-table embedding microbench (bench.py --roofline-only, roofline_aux
# embed_c5_bf16_microbench): product library vs the tools build (another revision of embed.hip)
set -o pipefail
mkdir -p gpurun_out
one() { timeout -k 10 200 $2 python bench.py --roofline-only > gpurun_out/eab.log 2>&1 || exit 1
        tail -1 gpurun_out/eab.log | python -c "
import json, sys
d = json.loads(sys.stdin.read())
for e in d['roofline_aux']:
    if e['kernel'] in ('embed_c5_bf16_microbench', 'embed_joint_fwd'):
        print('$1', e['kernel'], e['avg_ms'], e['achieved'], e.get('achieved_counter_GBs'))"; }
for i in 1 2 3; do one product ""; one tools "bash tools/with_tuning.sh"; done
