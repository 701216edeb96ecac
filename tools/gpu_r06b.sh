set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm_big or linear_fwd_act or linear_bwd or gemm_kernel or linear_f32" > gpurun_out/r06b_gemm_tests.log 2>&1 &&
timeout -k 10 200 python -u -m pytest tests/test_train_paths.py -m gpu -x -q --timeout 120 --timeout-method thread -k "held_across" > gpurun_out/r06b_ring.log 2>&1 &&
for v in 0 rule; do
  if [ $v = rule ]; then timeout -k 10 120 bash tools/with_tuning.sh python -u tools/gemm_big_bench.py; else timeout -k 10 120 bash tools/with_tuning.sh env ESGPT_GEMM_BIG=$v python -u tools/gemm_big_bench.py; fi || exit 1
done > gpurun_out/r06b_big_bench.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/r06b_gemm_tests.log; tail -2 gpurun_out/r06b_ring.log; cat gpurun_out/r06b_big_bench.log; exit $rc
