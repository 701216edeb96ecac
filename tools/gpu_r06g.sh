# Round-6 measurement set, part 1: C2 PMC traffic + bench line + step profile (tools/measure_config.sh), f32 line
set -o pipefail
mkdir -p gpurun_out
bash tools/measure_config.sh C2 20 > gpurun_out/r06g_measure_c2.log 2>&1 &&
timeout -k 10 300 python bench.py --dtype f32 --no-cpu-baseline > gpurun_out/r06g_bench_f32.log 2>&1
rc=$?; echo rc=$rc; tail -2 gpurun_out/r06g_measure_c2.log; grep '^{' gpurun_out/bench_C2.log | cut -c1-400; tail -1 gpurun_out/r06g_bench_f32.log | cut -c1-250; exit $rc
