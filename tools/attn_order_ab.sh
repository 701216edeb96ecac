# Workgroup order A/B of the attention kernels (ESGPT_ATTN_ORDER 0 / 1, tools build): fwd and bwd at the C2 / C3 /
# C5 / long layer shapes.
set -o pipefail
for m in 0 1; do
  ESGPT_ATTN_ORDER=$m timeout -k 10 200 bash tools/with_tuning.sh python tools/attn_time.py || { echo "FAILED $m"; exit 1; }
done
