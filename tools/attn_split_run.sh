set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "attention or width" > gpurun_out/attn_split_pytest.log 2>&1 || { tail -30 gpurun_out/attn_split_pytest.log; exit 1; }
tail -2 gpurun_out/attn_split_pytest.log
for m in 0 128 64; do
  ESGPT_ATTN_BWD_SPLIT2=$m timeout -k 10 200 bash tools/with_tuning.sh python tools/attn_split_ab.py || { echo "FAILED $m"; exit 1; }
done
python tools/attn_split_cmp.py gpurun_out/attn_split_0.pt gpurun_out/attn_split_128.pt gpurun_out/attn_split_64.pt | tail -3
