# Round-6 closing pass on the last tree: the whole GPU suite, smoke(), the C2 bench line (roofline + CPU baseline),
# C1 / C3 / C4 / C5 lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_pytest_gpu_close.log 2>&1 || { echo suite failed; grep -E "FAILED|Error" gpurun_out/r06_pytest_gpu_close.log | head; exit 1; }
tail -1 gpurun_out/r06_pytest_gpu_close.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r06_smoke_close.log 2>&1 || { echo smoke failed; tail gpurun_out/r06_smoke_close.log; exit 1; }
tail -1 gpurun_out/r06_smoke_close.log
timeout -k 10 300 python bench.py > gpurun_out/r06_bench_c2_close.log 2>&1 || { echo C2 failed; tail gpurun_out/r06_bench_c2_close.log; exit 1; }
grep '^{' gpurun_out/r06_bench_c2_close.log | cut -c1-200
for c in C1 C3 C4 C5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-roofline > gpurun_out/r06_bench_${c}_close.log 2>&1 || { echo $c failed; exit 1; }
  echo "$c $(grep '^{' gpurun_out/r06_bench_${c}_close.log | cut -c90-170)"
done
