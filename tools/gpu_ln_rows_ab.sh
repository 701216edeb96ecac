# LayerNorm rows per wave on the C2 step (tools build hooks ESGPT_LN_FWD_ROWS / ESGPT_LN_BWD_ROWS), alternating.
set -o pipefail
for i in 1 2; do
  for m in "" "ESGPT_LN_FWD_ROWS=2" "ESGPT_LN_BWD_ROWS=4"; do
    env $m timeout -k 10 200 bash tools/with_tuning.sh python bench.py --steps 40 --no-cpu-baseline --no-roofline --no-hbm-line > gpurun_out/ln.tmp 2>&1 || exit 1
    echo "${m:-default} $(grep '^{' gpurun_out/ln.tmp | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_step_median"])')" | tee -a gpurun_out/ln_rows_ab.log
  done
done
