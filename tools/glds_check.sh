#!/bin/bash
# LDS-DMA GEMM staging: parity (product build) then forward / backward timing per staging form (tools build).
#   gpurun -- bash tools/glds_check.sh
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "gemm or linear or mlp" tests/test_ops_gpu.py > gpurun_out/glds_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/glds_pytest.log
[ $rc -eq 0 ] || exit $rc
for f in 0 2 3; do
  echo "== forward, ESGPT_GEMM_FWD_GLDS=$f"
  ESGPT_GEMM_FWD_GLDS=$f timeout -k 10 120 bash tools/with_tuning.sh python -u tools/fwd_gemm_time.py || exit 1
done 2>&1 | tee gpurun_out/glds_fwd.log
for b in 0 2 3; do
  echo "== backward, ESGPT_GEMM_BWD_GLDS=$b"
  ESGPT_GEMM_BWD_GLDS=$b timeout -k 10 120 bash tools/with_tuning.sh python -u tools/bwd_pair_time.py || exit 1
done 2>&1 | tee gpurun_out/glds_bwd.log
