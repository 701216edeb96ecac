# One GPU call: the GPU suite, smoke, the default bench line and the f32 (reference-precision) bench line.
# usage: bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 \
  > gpurun_out/${TAG}_pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 &&
timeout -k 10 300 python bench.py --dtype f32 --no-cpu-baseline > gpurun_out/${TAG}_bench_f32.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/${TAG}_pytest_gpu.log; tail -2 gpurun_out/${TAG}_smoke.log
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400; tail -1 gpurun_out/${TAG}_bench_f32.log | cut -c1-400; exit $rc
