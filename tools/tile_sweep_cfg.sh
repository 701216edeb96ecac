# Step-time sweep of the GEMM tile hooks on one bench config (tools build): bash tools/tile_sweep_cfg.sh C4
set -o pipefail
cfg=${1:-C4}
run() {  # label, env
  env $2 timeout -k 10 200 bash tools/with_tuning.sh python bench.py --config $cfg --steps 10 --warmup 3 \
    --no-cpu-baseline --no-roofline --no-hbm-line 2>/dev/null | tail -1 | \
    python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['ms_per_step'], d['ms_per_step_median'])"
}
run default "ESGPT_X=0" || exit 1
for f in 21 22 12; do run "fwd=$f" "ESGPT_GEMM_TILE_FWD=$f" || exit 1; done
for x in 21 22; do run "dx=$x" "ESGPT_GEMM_TILE_DX=$x" || exit 1; done
run "dw=11" "ESGPT_GEMM_TILE_DW=11" || exit 1
run "dw=22" "ESGPT_GEMM_TILE_DW=22" || exit 1
run default "ESGPT_X=0" || exit 1
