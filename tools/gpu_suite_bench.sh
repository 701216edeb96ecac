#!/bin/bash
# Full GPU suite, then the default bench line (C2) — one GPU call.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread \
  > gpurun_out/suite.log 2>&1
rc=$?; tail -15 gpurun_out/suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; tail -3 gpurun_out/bench.log; exit $rc
