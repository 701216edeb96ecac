# Large-tile GEMM microbench (tools build): tools/gpu_bigbench.sh "0 rule"
set -o pipefail
mkdir -p gpurun_out
for v in ${1:-rule}; do
  if [ $v = rule ]; then timeout -k 10 120 bash tools/with_tuning.sh python -u tools/gemm_big_bench.py; else timeout -k 10 120 bash tools/with_tuning.sh env ESGPT_GEMM_BIG=$v python -u tools/gemm_big_bench.py; fi || exit 1
done > gpurun_out/bigbench.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/bigbench.log; exit $rc
