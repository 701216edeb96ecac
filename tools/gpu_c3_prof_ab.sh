set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 rule; do
  if [ $v = rule ]; then e=""; else e="ESGPT_GEMM_BIG=0"; fi
  timeout -k 10 200 bash tools/with_tuning.sh env $e rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3prof_$v -o run -- python bench.py --config C3 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-hbm-line > gpurun_out/c3prof_$v.log 2>&1 || exit 1
done
