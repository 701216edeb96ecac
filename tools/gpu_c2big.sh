# C2 projection shapes on the large-tile kernel's smaller tile configurations (tools build): parity, then timing
set -o pipefail
mkdir -p gpurun_out
run() { timeout -k 10 120 bash tools/with_tuning.sh env SQUARE=0 T=8192 D=256 F=1024 "$@" python -u tools/gemm_big_bench.py; }
{ timeout -k 10 300 bash tools/with_tuning.sh env ESGPT_GEMM_BIG=128 ESGPT_GEMM_BIG_TILE=64,128,4 ESGPT_GEMM_BIG_DWTILE=128,128,4 \
    python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "linear_bwd or test_gemm_kernel" &&
  run ESGPT_GEMM_BIG=0 &&
  run ESGPT_GEMM_BIG=128 ESGPT_GEMM_BIG_TILE=64,128,4 ESGPT_GEMM_BIG_DWTILE=128,128,4 &&
  run ESGPT_GEMM_BIG=128 ESGPT_GEMM_BIG_TILE=128,128,8 ESGPT_GEMM_BIG_DWTILE=128,128,8 &&
  run ESGPT_GEMM_BIG=128 ESGPT_GEMM_BIG_TILE=64,64,4 ESGPT_GEMM_BIG_DWTILE=64,128,4 &&
  run ESGPT_GEMM_BIG=128 ESGPT_GEMM_BIG_TILE=128,128,4 ESGPT_GEMM_BIG_DWTILE=128,256,8
} > gpurun_out/c2big.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/c2big.log | tail -32; exit $rc
