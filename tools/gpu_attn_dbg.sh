set -o pipefail
for nw in 0 8 0 8; do
  ESGPT_ATTN_FWD_NW=$nw timeout -k 10 100 bash tools/with_tuning.sh python tools/attn_dbg.py 2>&1 | grep -v amdgpu.ids
done
bash tools/attn_wide_tests.sh
