# GPU suite + C2 bench line + C3 step (bench + rocprof stats) + C2 step profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06d_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/r06d_bench_c2.log 2>&1 &&
timeout -k 10 300 python bench.py --config C3 --steps 10 --no-cpu-baseline --no-roofline > gpurun_out/r06d_bench_c3.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06d_step_c3 -o run -- \
    python bench.py --config C3 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-hbm-line > gpurun_out/r06d_step_c3.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06d_step_c2 -o run -- \
    python bench.py --config C2 --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-hbm-line > gpurun_out/r06d_step_c2.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/r06d_pytest_gpu.log
for f in c2 c3; do tail -1 gpurun_out/r06d_bench_$f.log | cut -c1-420; echo; done
exit $rc
