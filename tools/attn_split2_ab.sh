# Attention backward: fused kernel vs the split dK/dV + dQ pair (ESGPT_ATTN_BWD_SPLIT2 = 0 / 128 / 64, tools build)
# at the C2 / C3 / C5 / long shapes, then the attention parity tests with the split pair forced.
set -o pipefail
for sp in 0 128; do
  ESGPT_ATTN_BWD_SPLIT2=$sp ESGPT_ATTN_ORDER=split$sp timeout -k 10 200 bash tools/with_tuning.sh python tools/attn_time.py 2>&1 | grep -v amdgpu.ids || { echo "FAILED split=$sp"; exit 1; }
done
ESGPT_ATTN_BWD_SPLIT2=128 timeout -k 10 400 bash tools/with_tuning.sh python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread tests/test_gpu_parity.py tests/test_ops_gpu.py -k "attention" -m gpu > gpurun_out/attn_split2_tests.log 2>&1 || { echo "TESTS FAILED split"; grep -E "FAILED|Error|assert" gpurun_out/attn_split2_tests.log | head; exit 1; }
echo "tests split=128: $(tail -1 gpurun_out/attn_split2_tests.log)"
