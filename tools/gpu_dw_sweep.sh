set -o pipefail
mkdir -p gpurun_out
for t in 0 64 128 256 768 1024 2048; do
  echo "== ESGPT_GEMM_DW_TARGET=$t"; timeout -k 10 100 bash tools/with_tuning.sh env ESGPT_GEMM_DW_TARGET=$t python tools/bwd_pair_time.py 2>&1 | grep -v amdgpu || exit 1
done > gpurun_out/dw_sweep.log 2>&1
rc=$?; cat gpurun_out/dw_sweep.log; exit $rc
