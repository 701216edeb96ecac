#!/bin/bash
# f32 MFMA attention: parity tests (kernel shapes, dropout, f32 goldens), then the f32 C2 step's kernel stats.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/af32
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_ops_gpu.py -k "attention or golden or f32 or width" > gpurun_out/af32/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/af32/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/af32/pytest.log | head -20; exit $rc; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/af32/prof -o run -- \
  python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --dtype f32 > gpurun_out/af32/bench.log 2>&1 || exit 2
f=$(find gpurun_out/af32/prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/af32/kernel_stats.csv
find gpurun_out/af32/prof -name "*.csv" -delete
python3 tools/prof_summary.py gpurun_out/af32/kernel_stats.csv - 25
grep '^{' gpurun_out/af32/bench.log | cut -c1-200
