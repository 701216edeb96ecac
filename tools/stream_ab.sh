# A/B of the streamed-tile GEMM configurations against the tile GEMM (tools build), one process per setting.
set -o pipefail
mkdir -p gpurun_out
for m in 0 223 222 214 213 124 114; do
  ESGPT_GEMM_STREAM=$m timeout -k 10 120 bash tools/with_tuning.sh python tools/stream_check.py || { echo "FAILED mode $m"; exit 1; }
done
