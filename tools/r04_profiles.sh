#!/bin/bash
# Round-4 evidence in one GPU call: the f32 (reference-precision) C2 bench line, and rocprofv3 kernel stats of the
# C2 f32, C2 bf16 and C4 bf16 steps (graph replay).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --dtype f32 > gpurun_out/r04/bench_c2_f32.log 2>&1 || exit 1
for spec in "c2_f32:--dtype f32" "c2_bf16:" "c4_bf16:--config C4"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04/$name -o run -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline $args > gpurun_out/r04/$name.log 2>&1 || exit 2
  f=$(find gpurun_out/r04/$name -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/r04/${name}_kernel_stats.csv
  python3 tools/prof_summary.py gpurun_out/r04/${name}_kernel_stats.csv - 60 > gpurun_out/r04/${name}_summary.txt
  find gpurun_out/r04/$name -name "*.csv" ! -name "*kernel_stats.csv" -delete
done
tail -1 gpurun_out/r04/bench_c2_f32.log | cut -c1-300
