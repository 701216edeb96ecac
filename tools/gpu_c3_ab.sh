# C3 step A/B on one box: tile GEMM (ESGPT_GEMM_BIG=0) vs the product rule, alternating (tools build)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in 0 rule; do
    if [ $v = rule ]; then e=""; else e="ESGPT_GEMM_BIG=0"; fi
    timeout -k 10 200 bash tools/with_tuning.sh env $e python bench.py --config ${CFG:-C3} --steps 10 --no-cpu-baseline --no-roofline --no-hbm-line > gpurun_out/c3ab.log 2>&1 || exit 1
    echo "big=$v $(grep '^{' gpurun_out/c3ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_step_median"])')"
  done
done
