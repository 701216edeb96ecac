# End-of-round GPU pass (one call): the GPU suite, smoke, C2's measurement set (PMC traffic, bench line, step
# profile), the f32 bench line. Stops at the first failure.
set -o pipefail
TAG=${1:-r05}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 \
  > gpurun_out/${TAG}_pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 &&
bash tools/measure_config.sh C2 20 > gpurun_out/${TAG}_measure_c2.log 2>&1 &&
timeout -k 10 300 python bench.py --dtype f32 --no-cpu-baseline > gpurun_out/${TAG}_bench_f32.log 2>&1
rc=$?
echo "rc=$rc"; tail -3 gpurun_out/${TAG}_pytest_gpu.log; tail -2 gpurun_out/${TAG}_smoke.log
tail -1 gpurun_out/bench_C2.log | cut -c1-300; tail -1 gpurun_out/${TAG}_bench_f32.log | cut -c1-300
exit $rc
