set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm_big or linear_fwd_act or linear_bwd" > gpurun_out/r06c_gemm_tests.log 2>&1 &&
bash tools/gpu_bigbench.sh rule && bash tools/gpu_pmc_square.sh
rc=$?; tail -2 gpurun_out/r06c_gemm_tests.log; exit $rc
