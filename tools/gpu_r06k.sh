# Split backward at hd 64 (with dropout too): the whole GPU suite, then C2 / C3 / C5 bench lines.
set -o pipefail
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06k_pytest.log 2>&1 || { echo suite failed; grep -E "FAILED|Error" gpurun_out/r06k_pytest.log | head; tail -3 gpurun_out/r06k_pytest.log; exit 1; }
tail -1 gpurun_out/r06k_pytest.log
for c in C2 C3 C5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-roofline > gpurun_out/r06k_bench_$c.log 2>&1 || { echo $c failed; exit 1; }
  echo "$c $(grep '^{' gpurun_out/r06k_bench_$c.log | cut -c90-160)"
done
