# Wide attention forward A/B (ESGPT_ATTN_FWD_NW = 0 parity form / 4 / 8 waves, tools build) at the C2 / C3 / C5 /
# long layer shapes, then the attention parity tests with each wide form forced on every hd-64 shape.
set -o pipefail
for nw in 0 4 8; do
  ESGPT_ATTN_FWD_NW=$nw timeout -k 10 200 bash tools/with_tuning.sh python tools/attn_time.py \
    || { echo "FAILED nw=$nw"; exit 1; }
done
for nw in 0 4 8; do
  ESGPT_ATTN_FWD_NW=$nw timeout -k 10 400 bash tools/with_tuning.sh python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread tests/test_gpu_parity.py -k "attention_kernel or attention_dropout" -m gpu \
    > gpurun_out/attn_wide_tests_nw$nw.log 2>&1 || { echo "TESTS FAILED nw=$nw"; tail -30 gpurun_out/attn_wide_tests_nw$nw.log; exit 1; }
  echo "tests nw=$nw: $(tail -1 gpurun_out/attn_wide_tests_nw$nw.log)"
done
