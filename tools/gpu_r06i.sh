# Attention parity (product rule + forced wide forms), then the C2 bench line and the C3 / C5 step times.
set -o pipefail
bash tools/attn_wide_tests.sh || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r06i_bench_c2.log 2>&1 || { echo bench failed; tail gpurun_out/r06i_bench_c2.log; exit 1; }
grep '^{' gpurun_out/r06i_bench_c2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("C2", d["value"], d["ms_per_step"]); [print(a["kernel"], a["avg_ms"], round(a["frac"],4)) for a in d["roofline_aux"]]'
for c in C3 C5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-roofline --no-hbm-line > gpurun_out/r06i_bench_$c.log 2>&1 || { echo bench $c failed; exit 1; }
  echo "$c $(grep '^{' gpurun_out/r06i_bench_$c.log | cut -c1-200)"
done
