# Round-6 final pass, part 1: the whole GPU suite, then smoke().
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 > gpurun_out/r06_pytest_gpu_final.log 2>&1 &&
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r06_smoke_final.log 2>&1
rc=$?; echo "rc=$rc"; tail -4 gpurun_out/r06_pytest_gpu_final.log; tail -3 gpurun_out/r06_smoke_final.log; exit $rc
