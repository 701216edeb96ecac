# Embedding forward with a wave-level instead of a workgroup barrier (tools build) vs the product build: the bench's
# isolated embedding entries, then C5 / C2 steps, alternating on one box; then the embedding parity tests (tools).
set -o pipefail
for i in 1 2; do
  for m in prod wave; do
    if [ $m = prod ]; then
      timeout -k 10 200 python bench.py --roofline-only > gpurun_out/es.tmp 2>&1 || exit 1
    else
      timeout -k 10 200 bash tools/with_tuning.sh python bench.py --roofline-only > gpurun_out/es.tmp 2>&1 || exit 1
    fi
    echo "$m $(grep '^{' gpurun_out/es.tmp | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print([(a["kernel"], a["avg_ms"]) for a in d["roofline_aux"] if a["kernel"].startswith("embed")])')" | tee -a gpurun_out/embed_sync_ab.log
  done
done
for c in C5 C2; do
  for m in prod wave prod wave; do
    if [ $m = prod ]; then
      timeout -k 10 200 python bench.py --config $c --steps 30 --no-cpu-baseline --no-roofline --no-hbm-line > gpurun_out/es.tmp 2>&1 || exit 1
    else
      timeout -k 10 200 bash tools/with_tuning.sh python bench.py --config $c --steps 30 --no-cpu-baseline --no-roofline --no-hbm-line > gpurun_out/es.tmp 2>&1 || exit 1
    fi
    echo "$c $m $(grep '^{' gpurun_out/es.tmp | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_step_median"])')" | tee -a gpurun_out/embed_sync_ab.log
  done
done
timeout -k 10 400 bash tools/with_tuning.sh python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "embed" > gpurun_out/embed_sync_tests.log 2>&1 || { echo tests failed; tail -20 gpurun_out/embed_sync_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/embed_sync_tests.log)"
