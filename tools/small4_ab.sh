# A/B of the small4 attention items per wave (tools build): one process per ESGPT_SMALL4_NI value ("fwd,bwd")
set -o pipefail
for ni in 1,1 2,2 2,1 1,2 2,2; do
  ESGPT_SMALL4_NI=$ni timeout -k 10 120 bash tools/with_tuning.sh python tools/small4_time.py || exit 1
done
