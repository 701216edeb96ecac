#!/bin/bash
# C2 bench under tuning-hook settings, one process each, in one GPU session: tools/env_sweep.sh "ENV=..;ENV2=.." ...
# ("-" = defaults). Prints ms/step (mean, median) per setting. Needs the tools build of the library: `make -C
# eventstreamgpt_amd/csrc TUNING=1` (the product build ignores these variables; rebuild with plain make afterwards).
for spec in "$@"; do
  envs=()
  if [ "$spec" != "-" ]; then IFS=';' read -ra envs <<< "$spec"; fi
  out=$(env "${envs[@]}" timeout -k 10 120 python bench.py --config ${CONFIG:-C2} --steps ${STEPS:-100} --warmup 10 --no-roofline --no-cpu-baseline --no-hbm-line 2>/dev/null | grep '^{')
  rc=$?
  if [ $rc -ne 0 ]; then echo "$spec: failed rc=$rc"; exit $rc; fi
  echo "$spec: $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_step_median"])')"
done
