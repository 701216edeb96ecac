# Fused vs split attention backward with right-padded key masks (PAD=1), tools build.
set -o pipefail
for sp in 0 128; do
  PAD=1 ESGPT_ATTN_BWD_SPLIT2=$sp ESGPT_ATTN_ORDER=pad-split$sp timeout -k 10 200 bash tools/with_tuning.sh python tools/attn_time.py 2>&1 | grep -v amdgpu.ids || exit 1
done
