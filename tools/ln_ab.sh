# Same-box A/B: product library vs the tools build (built from another revision of a kernel source), LN microbench
set -o pipefail
for i in 1 2 3; do
  echo "product:"; timeout -k 10 120 python tools/ln_bench.py 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
  echo "tools build:"; timeout -k 10 120 bash tools/with_tuning.sh python tools/ln_bench.py 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
done
