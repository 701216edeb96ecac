# The attention parity tests with the wide forward forced off / 4 / 8 waves (tools build), then on the product build.
set -o pipefail
for nw in 0 4 8; do
  ESGPT_ATTN_FWD_NW=$nw timeout -k 10 400 bash tools/with_tuning.sh python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread tests/test_gpu_parity.py tests/test_ops_gpu.py -k "attention" -m gpu \
    > gpurun_out/attn_wide_tests_nw$nw.log 2>&1 || { echo "TESTS FAILED nw=$nw"; grep -E "FAILED|Error|assert" gpurun_out/attn_wide_tests_nw$nw.log | head -20; exit 1; }
  echo "tests nw=$nw: $(tail -1 gpurun_out/attn_wide_tests_nw$nw.log)"
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_ops_gpu.py -k "attention" -m gpu > gpurun_out/attn_tests_prod.log 2>&1 || { echo "PRODUCT TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/attn_tests_prod.log | head; exit 1; }
echo "product: $(tail -1 gpurun_out/attn_tests_prod.log)"
