# Round-6 final pass, part 2: the C2 bench line (roofline + CPU baseline), C1 / C3 / C4 / C5 lines, the C2 step
# profile (rocprofv3 kernel stats).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/r06_bench_c2_final.log 2>&1 || { echo C2 failed; tail gpurun_out/r06_bench_c2_final.log; exit 1; }
grep '^{' gpurun_out/r06_bench_c2_final.log | cut -c1-330
for c in C1 C3 C4 C5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-roofline > gpurun_out/r06_bench_${c}_final.log 2>&1 || { echo $c failed; tail gpurun_out/r06_bench_${c}_final.log; exit 1; }
  grep '^{' gpurun_out/r06_bench_${c}_final.log | cut -c1-200
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/step_C2_final -o run -- \
    python bench.py --steps 25 --warmup 3 --no-cpu-baseline --no-roofline --no-hbm-line > gpurun_out/step_C2_final.log 2>&1 || { echo profile failed; exit 1; }
echo done
