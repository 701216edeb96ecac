#!/bin/bash
# Attention parity + timing on the GPU box: the attention GPU tests (op vs C ABI, keep bits vs re-hash, parity vs
# torch f32 with the keep mask replayed), then the C2 attention roofline entries.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "attention or attn" > gpurun_out/pytest_attn.log 2>&1 &&
timeout -k 10 200 python tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_attn.log
cat gpurun_out/attn_bench.log | tail -20
exit $rc
