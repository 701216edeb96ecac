# Same-box A/B of the dependency-graph row-block skipping on the C4 step (tools build for the IGNORE variant):
# on / python off / python on but kernels ignore the mask
set -o pipefail
run() {  # label, env, args
  env $2 timeout -k 10 300 bash tools/with_tuning.sh python bench.py --config C4 --no-cpu-baseline --no-roofline $3 \
    2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['ms_per_step'], d['ms_per_step_median'])"
}
for rep in 1 2; do
  run on "ESGPT_X=0" "--row-tiles" || exit 1
  run off "ESGPT_X=0" "" || exit 1
  run ignore "ESGPT_ROW_TILES_IGNORE=1" "--row-tiles" || exit 1
done
