set -o pipefail
mkdir -p gpurun_out
{ timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm_big or linear_fwd_act or linear_bwd" &&
  for c in 1024 2048 512; do timeout -k 10 120 bash tools/with_tuning.sh env SQUARE=0 ESGPT_GEMM_BIG_DWCHUNK=$c python -u tools/gemm_big_bench.py || exit 1; done
} > gpurun_out/bigbench3.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/bigbench3.log | tail -17; exit $rc
