# Same-box A/B: product library vs the tools build (another revision of losses.hip), C2 loss microbench (stream path)
set -o pipefail
for i in 1 2 3; do
  echo "product:"; LOSS_BENCH_ONLY=all timeout -k 10 120 python tools/loss_bench.py 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-200 || exit 1
  echo "tools build:"; LOSS_BENCH_ONLY=all timeout -k 10 120 bash tools/with_tuning.sh python tools/loss_bench.py 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-200 || exit 1
done
