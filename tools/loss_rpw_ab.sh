# A/B of the streaming loss kernel's rows per wave (tools build): C2 output_loss timing per ESGPT_LOSS_RPW value
set -o pipefail
for r in 1 2 4 1 2; do
  echo "rpw=$r"
  ESGPT_LOSS_RPW=$r LOSS_BENCH_ONLY=all timeout -k 10 120 bash tools/with_tuning.sh python tools/loss_bench.py 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
done
