# Timing half of tools/attn_wide_ab.sh: fwd / bwd at the C2 / C3 / C5 / long shapes, parity form vs 4 / 8 waves.
set -o pipefail
for nw in 0 4 8; do
  ESGPT_ATTN_FWD_NW=$nw timeout -k 10 200 bash tools/with_tuning.sh python tools/attn_time.py 2>&1 | grep -v amdgpu.ids \
    || { echo "FAILED nw=$nw"; exit 1; }
done
