# Step-level A/B of the split attention backward at hd 64 (tools build: ESGPT_ATTN_BWD_SPLIT2=0 forces the fused
# kernel; unset = the product rule), alternating on one box, C3 and C5.
set -o pipefail
for c in C5 C3; do
  for i in 1 2; do
    for m in rule 0; do
      if [ $m = rule ]; then
        timeout -k 10 200 bash tools/with_tuning.sh python bench.py --config $c --steps 30 --no-cpu-baseline --no-roofline --no-hbm-line > gpurun_out/ab.tmp 2>&1 || exit 1
      else
        ESGPT_ATTN_BWD_SPLIT2=0 timeout -k 10 200 bash tools/with_tuning.sh python bench.py --config $c --steps 30 --no-cpu-baseline --no-roofline --no-hbm-line > gpurun_out/ab.tmp 2>&1 || exit 1
      fi
      echo "$c split=$m $(grep '^{' gpurun_out/ab.tmp | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_step_median"])')" | tee -a gpurun_out/split_step_ab.log
    done
  done
done
