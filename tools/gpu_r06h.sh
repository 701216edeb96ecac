# Error words through mapped host memory: error / train-path GPU tests, then C2 A/B against the per-step D2H copy
# (--err-copy), alternating, PCIe-inclusive value.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_errors_gpu.py \
  tests/test_train_paths.py -m gpu > gpurun_out/r06h_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r06h_tests.log; exit 1; }
tail -2 gpurun_out/r06h_tests.log
for i in 1 2 3; do
  for m in "" "--err-copy"; do
    timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-roofline --no-cpu-baseline --no-hbm-line $m \
      > gpurun_out/r06h_ab.tmp 2>&1 || { echo bench failed; tail -20 gpurun_out/r06h_ab.tmp; exit 1; }
    echo "${m:-hostwords} $(grep '^{' gpurun_out/r06h_ab.tmp | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_step_median"])')" | tee -a gpurun_out/r06h_ab.log
  done
done
