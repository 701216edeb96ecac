# Wide attention forward: 1 vs 2 query slices per wave (ESGPT_ATTN_FWD_NU, 4 waves forced), timing + parity tests.
set -o pipefail
for nu in 1 2; do
  ESGPT_ATTN_FWD_NW=4 ESGPT_ATTN_FWD_NU=$nu ESGPT_ATTN_ORDER=nu$nu timeout -k 10 200 bash tools/with_tuning.sh python tools/attn_time.py 2>&1 | grep -v amdgpu.ids || { echo "FAILED nu=$nu"; exit 1; }
done
ESGPT_ATTN_FWD_NW=4 ESGPT_ATTN_FWD_NU=2 timeout -k 10 400 bash tools/with_tuning.sh python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread tests/test_gpu_parity.py tests/test_ops_gpu.py -k "attention" -m gpu > gpurun_out/attn_nu2_tests.log 2>&1 || { echo "TESTS FAILED nu=2"; grep -E "FAILED|Error|assert" gpurun_out/attn_nu2_tests.log | head; exit 1; }
echo "tests nu=2: $(tail -1 gpurun_out/attn_nu2_tests.log)"
