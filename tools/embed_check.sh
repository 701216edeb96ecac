#!/bin/bash
# Embedding parity (bag backward vs float64, bitwise repeats, known answers, model parity) and the backward's
# per-kernel split at the C2 / C5 batches.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_embed_bwd_gpu.py tests/test_embedding_known_answers_gpu.py \
    tests/test_gpu_parity.py tests/test_errors_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_embed.log 2>&1 &&
timeout -k 10 120 python tools/embed_bwd_bench.py > gpurun_out/embed_bwd_bench.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/embprof -o run -- \
    python tools/embed_bwd_bench.py > /dev/null 2>&1
rc=$?
tail -2 gpurun_out/pytest_embed.log
grep -v amdgpu.ids gpurun_out/embed_bwd_bench.log
exit $rc
