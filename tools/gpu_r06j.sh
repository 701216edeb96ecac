# Split backward at hd 64 (no dropout) in the product: attention parity tests, then the C2 measurement set (PMC
# traffic incl. the long-sequence attention entries, bench line, step profile).
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_ops_gpu.py -k "attention" -m gpu > gpurun_out/r06j_tests.log 2>&1 || { echo tests failed; tail -20 gpurun_out/r06j_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r06j_tests.log)"
bash tools/measure_config.sh C2 20 > gpurun_out/r06j_measure.log 2>&1 || { echo measure failed; tail gpurun_out/r06j_measure.log; exit 1; }
grep '^{' gpurun_out/bench_C2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("C2", d["value"], d["ms_per_step"], d["roofline"]["frac"]); [print(a["kernel"], a["symbol"], a["avg_ms"], round(a["frac"],4), a.get("traffic")) for a in d["roofline_aux"]]'
