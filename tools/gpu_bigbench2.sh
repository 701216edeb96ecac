# tools/gpu_bigbench2.sh: C3 under the product rule / 6 ring slots, and C2's shapes forced onto the large tiles
set -o pipefail
mkdir -p gpurun_out
{ timeout -k 10 120 bash tools/with_tuning.sh env SQUARE=0 ESGPT_GEMM_BIG_SLOTS=6 python -u tools/gemm_big_bench.py &&
  for v in 0 128 256; do timeout -k 10 120 bash tools/with_tuning.sh env SQUARE=0 T=8192 D=256 F=1024 ESGPT_GEMM_BIG=$v python -u tools/gemm_big_bench.py || exit 1; done
} > gpurun_out/bigbench2.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/bigbench2.log; exit $rc
