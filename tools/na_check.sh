#!/bin/bash
# NA glue on the GPU box: the new op tests, the NA parity / train-path tests, then the C4 bench step time.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_gpu_parity.py tests/test_train_paths.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_na.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_na.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/bench_C4_na.log 2>&1
rc=$?
tail -1 gpurun_out/bench_C4_na.log | cut -c1-300
exit $rc
