# Step-level A/B of the wide attention forward on C3 (tools build: ESGPT_ATTN_FWD_NW=0 forces the parity form; unset =
# the product rule), alternating on one box; then the attention parity tests on the product build.
set -o pipefail
for i in 1 2; do
  for m in rule 0; do
    if [ $m = rule ]; then
      timeout -k 10 200 bash tools/with_tuning.sh python bench.py --config C3 --steps 30 --no-cpu-baseline --no-roofline --no-hbm-line > gpurun_out/ab.tmp 2>&1 || exit 1
    else
      ESGPT_ATTN_FWD_NW=0 timeout -k 10 200 bash tools/with_tuning.sh python bench.py --config C3 --steps 30 --no-cpu-baseline --no-roofline --no-hbm-line > gpurun_out/ab.tmp 2>&1 || exit 1
    fi
    echo "C3 wide=$m $(grep '^{' gpurun_out/ab.tmp | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_step_median"])')" | tee -a gpurun_out/wide_step_ab.log
  done
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_ops_gpu.py -k "attention" -m gpu > gpurun_out/r06l_tests.log 2>&1 || { echo tests failed; tail -20 gpurun_out/r06l_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r06l_tests.log)"
