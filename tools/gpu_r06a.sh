set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 > gpurun_out/r06a_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/r06a_bench.log 2>&1
rc=$?; echo "rc=$rc"; tail -5 gpurun_out/r06a_pytest_gpu.log; tail -1 gpurun_out/r06a_bench.log | cut -c1-700; exit $rc
